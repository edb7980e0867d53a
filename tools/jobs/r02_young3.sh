# young-wave cutoff (S >= 64 variants, cutoff 8) against the previous build over the large profiles.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_young
mkdir -p $O
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/y0/libmsv_hip.so ab/yn/libmsv_hip.so > $O/ab3.jsonl
for p in 1001.hmm 1200.hmm 1600.hmm 1901.hmm 2138.hmm; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile $p --rounds 2 --warm 8 --time 10 ab/y0/libmsv_hip.so ab/yn/libmsv_hip.so >> $O/ab3.jsonl
done
timeout -k 10 300 python tools/kernel_ab.py --config cfg5 --rounds 2 --warm 3 --time 4 ab/y0/libmsv_hip.so ab/yn/libmsv_hip.so >> $O/ab3.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg4 --rounds 2 --warm 2 --time 3 ab/y0/libmsv_hip.so ab/yn/libmsv_hip.so >> $O/ab3.jsonl
