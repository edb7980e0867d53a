# (experiment) young-wave cutoff, second A/B: larger cutoffs on cfg3 and cfg4-sized batch.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_young
mkdir -p $O
timeout -k 10 500 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/y0/libmsv_hip.so ab/y8/libmsv_hip.so ab/y12/libmsv_hip.so ab/y16/libmsv_hip.so > $O/ab2.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 2 ab/y0/libmsv_hip.so ab/y8/libmsv_hip.so ab/y16/libmsv_hip.so >> $O/ab2.jsonl
