# Residue blocks for long rows (8 or 16 rows per block) vs one byte per row: kernel A/B on cfg3 and 900.hmm.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_blkl
mkdir -p $O
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/cur/libmsv_hip.so ab/blkl8/libmsv_hip.so ab/blkl16/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 900.hmm --rounds 2 ab/cur/libmsv_hip.so ab/blkl8/libmsv_hip.so ab/blkl16/libmsv_hip.so > $O/ab_900.jsonl
