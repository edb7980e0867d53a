# Round 4, first GPU pass: the Viterbi stage's GPU tests, the clock-stamp A/B (cfg3, cfg2), then the
# whole GPU suite (grid ADVICE fixes, cfg4/cfg5 every score).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_vit1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/base/libmsv_hip.so ab/stamp/libmsv_hip.so > $O/ab_stamp_cfg3.jsonl 2> $O/ab_stamp.err
timeout -k 10 200 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/stamp/libmsv_hip.so > $O/ab_stamp_cfg2.jsonl 2>> $O/ab_stamp.err
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_viterbi.py > $O/pytest_gpu.log 2>&1
