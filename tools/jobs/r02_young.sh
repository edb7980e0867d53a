# (experiment) youngest-quarter waves stop taking sequences near the end of the queue: cfg3 kernel A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_young
mkdir -p $O
export MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/y4/libmsv_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "full_size or homolog or seeded" --timeout 240 --timeout-method thread > $O/pytest_y4.log 2>&1
unset MSV_LIB_PATH
timeout -k 10 500 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/y0/libmsv_hip.so ab/y2/libmsv_hip.so ab/y4/libmsv_hip.so ab/y8/libmsv_hip.so > $O/ab.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg5 --rounds 1 --warm 3 --time 4 ab/y0/libmsv_hip.so ab/y4/libmsv_hip.so >> $O/ab.jsonl
