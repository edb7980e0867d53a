# Next-row ring prefetch for long rows (XNEXT): parity on the forced variants, kernel A/B on cfg3 and 1001/1901.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_xn
mkdir -p $O
export MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/xn1/libmsv_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
unset MSV_LIB_PATH
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/xn0/libmsv_hip.so ab/xn1/libmsv_hip.so > $O/ab.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 1001.hmm --rounds 2 ab/xn0/libmsv_hip.so ab/xn1/libmsv_hip.so >> $O/ab.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 1901.hmm --rounds 2 ab/xn0/libmsv_hip.so ab/xn1/libmsv_hip.so >> $O/ab.jsonl
