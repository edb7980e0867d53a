# Round 6: record the speed gate's table at HEAD's kernels, then the gate against it (HEAD) and against the
# pre-30adc47 build (round 5's 40x Viterbi regression: must fail).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_g
mkdir -p $O
SPEED_GATE_RECORD=$O/speed_table.json timeout -k 10 120 python -u -m pytest tests/test_speed_gate.py -m gpu -x -q -s --timeout 100 --timeout-method thread > $O/speed_gate_record.log 2>&1
cp $O/speed_table.json tests/golden/speed_table.json
timeout -k 10 120 python -u -m pytest tests/test_speed_gate.py -m gpu -x -q -s --timeout 100 --timeout-method thread --durations=1 > $O/speed_gate_head.log 2>&1
MSV_LIB_PATH=$PWD/abx/pre30adc47/libmsv_hip.so timeout -k 10 120 python -u -m pytest tests/test_speed_gate.py -m gpu -x -q -s --timeout 100 --timeout-method thread --durations=1 > $O/speed_gate_pre30adc47.log 2>&1 || echo "gate rc=$? on pre30adc47" >> $O/speed_gate_pre30adc47.log
