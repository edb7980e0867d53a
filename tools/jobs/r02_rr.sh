# Static first assignment dealt by SIMD rounds (ab/rr) vs contiguous (ab/base) vs per-group interleave (ab/il).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_rr
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/il/libmsv_hip.so ab/rr/libmsv_hip.so > $O/ab.jsonl
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/base/libmsv_hip.so ab/il/libmsv_hip.so ab/rr/libmsv_hip.so >> $O/ab.jsonl
for n in 2048 8192; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --n $n --rounds 2 --warm 5 --time 10 ab/base/libmsv_hip.so ab/il/libmsv_hip.so ab/rr/libmsv_hip.so >> $O/ab.jsonl
done
for n in 256 2048; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 1901.hmm --n $n --rounds 2 --warm 3 --time 5 ab/base/libmsv_hip.so ab/il/libmsv_hip.so ab/rr/libmsv_hip.so >> $O/ab.jsonl
done
timeout -k 10 300 python tools/kernel_ab.py --config cfg5 --rounds 1 --warm 3 --time 4 ab/base/libmsv_hip.so ab/rr/libmsv_hip.so >> $O/ab.jsonl
