set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_xn2
mkdir -p $O
for p in 1301.hmm 1509.hmm 1200.hmm; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile $p --rounds 2 ab/xn0/libmsv_hip.so ab/xn1/libmsv_hip.so >> $O/ab.jsonl
done
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 2 ab/xn0/libmsv_hip.so ab/xn1/libmsv_hip.so >> $O/ab.jsonl
