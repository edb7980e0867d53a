set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_rr2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/base/libmsv_hip.so ab/rr2/libmsv_hip.so > $O/ab.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --n 4096 --rounds 2 --warm 5 --time 10 ab/base/libmsv_hip.so ab/rr2/libmsv_hip.so >> $O/ab.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 2 ab/base/libmsv_hip.so ab/rr2/libmsv_hip.so >> $O/ab.jsonl
