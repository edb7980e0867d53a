# (experiment) deeper residue prefetch for long rows (S > 40): zero-copy (pinned host residues) vs HBM kernel time.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_rpf
mkdir -p $O
for r in 1 2 3 1 2 3; do
  MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/rpf$r/libmsv_hip.so timeout -k 10 200 python tools/zero_copy_probe.py --config cfg3 --time 10 | sed "s/^{/{\"rpf\": $r, /" >> $O/zc.jsonl
done
MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/rpf3/libmsv_hip.so timeout -k 10 200 python tools/zero_copy_probe.py --config cfg5 --time 4 | sed "s/^{/{\"rpf\": 3, /" >> $O/zc.jsonl
MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/rpf1/libmsv_hip.so timeout -k 10 200 python tools/zero_copy_probe.py --config cfg5 --time 4 | sed "s/^{/{\"rpf\": 1, /" >> $O/zc.jsonl
