# Round 6: (1) whole GPU suite at the working tree (team exchange as one combined record with per-half stamps,
# O(n) survivor scan, clamp, short-row combined J/event test); (2) the speed gate's table recorded; (3) the gate
# against the pre-30adc47 build (must fail); (4) interleaved A/Bs: team picks cfg5 / cfg3 vs HEAD~ (r6base ->
# r6x1), cfg2 kernel + one-wave row time: r6x1 (base) / r6x2 (combined test) / r6x3 (+ sameEJ assumed, timing-only).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_speed_gate.py > $O/pytest_gpu.log 2>&1
SPEED_GATE_RECORD=$O/speed_table.json timeout -k 10 120 python -u -m pytest tests/test_speed_gate.py -m gpu -x -q -s --timeout 100 --timeout-method thread > $O/speed_gate_record.log 2>&1 || true
cp $O/speed_table.json tests/golden/speed_table.json
MSV_LIB_PATH=$PWD/abx/pre30adc47/libmsv_hip.so timeout -k 10 120 python -u -m pytest tests/test_speed_gate.py -m gpu -x -q -s --timeout 100 --timeout-method thread > $O/speed_gate_pre30adc47.log 2>&1 || echo "gate rc=$? on pre30adc47" >> $O/speed_gate_pre30adc47.log
timeout -k 10 240 python -u tools/kernel_ab.py --config cfg2 --rounds 4 abx/r6x1/libmsv_hip.so abx/r6x2/libmsv_hip.so abx/r6x3/libmsv_hip.so > $O/ab_cfg2.jsonl 2> $O/ab_cfg2.err
for L in r6x1 r6x2 r6x3; do MSV_LIB_PATH=$PWD/abx/$L/libmsv_hip.so timeout -k 10 60 python -u tools/cfg2_floor.py > $O/floor_$L.json 2>> $O/floor.err; done
for L in r6seg0 r6seg; do MSV_LIB_PATH=$PWD/abx/$L/libmsv_hip.so timeout -k 10 90 python -u tools/cfg2_segments.py > $O/segments_$L.jsonl 2>> $O/segments.err; done
timeout -k 10 240 python -u tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 2 --in-place abx/r6base/libmsv_hip.so abx/r6x1/libmsv_hip.so > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err
timeout -k 10 150 python -u tools/vit_ab.py --config cfg3 --variant vit_w1_s22_ea --rounds 2 --in-place abx/r6base/libmsv_hip.so abx/r6x1/libmsv_hip.so > $O/ab_cfg3.jsonl 2> $O/ab_cfg3.err
