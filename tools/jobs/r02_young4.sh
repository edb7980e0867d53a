# graded young-wave cutoffs per quarter of the block's waves (Q1/Q2/Q3 in n_groups/4 units).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_young
mkdir -p $O
L="ab/yn/libmsv_hip.so ab/q008/libmsv_hip.so ab/q028/libmsv_hip.so ab/q048/libmsv_hip.so ab/q248/libmsv_hip.so ab/q0412/libmsv_hip.so"
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 $L > $O/ab4.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 1001.hmm --rounds 2 --warm 8 --time 10 $L >> $O/ab4.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg5 --rounds 1 --warm 3 --time 4 $L >> $O/ab4.jsonl
