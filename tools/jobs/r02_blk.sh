# Residue blocks (BLK) for short rows: GPU parity suite, then interleaved kernel A/B against HEAD's build
# on cfg2 (100.hmm x 10k), a small-profile throughput batch (400.hmm x 100k) and the 1400.hmm latency
# plan (2048 sequences).  Needs ab/base (bash tools/ab_build.sh HEAD base) and ab/blk (. blk).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_blk
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 4 ab/base/libmsv_hip.so ab/blk/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --profile 400.hmm --n 100000 --rounds 3 ab/base/libmsv_hip.so ab/blk/libmsv_hip.so > $O/ab_400_100k.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --n 2048 --rounds 3 ab/base/libmsv_hip.so ab/blk/libmsv_hip.so > $O/ab_1400_2048.jsonl
