# (experiment) residue prefetch 2 rows ahead for long rows: resident (HBM) kernel A/B on cfg3, 1001.hmm, 1901.hmm, cfg5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_rpf
mkdir -p $O
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 4 ab/rpf1/libmsv_hip.so ab/rpf2/libmsv_hip.so > $O/ab_hbm.jsonl
for p in 1001.hmm 1901.hmm; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile $p --rounds 2 --warm 8 --time 10 ab/rpf1/libmsv_hip.so ab/rpf2/libmsv_hip.so >> $O/ab_hbm.jsonl
done
timeout -k 10 300 python tools/kernel_ab.py --config cfg5 --rounds 2 --warm 3 --time 4 ab/rpf1/libmsv_hip.so ab/rpf2/libmsv_hip.so >> $O/ab_hbm.jsonl
