# Order kernels A/B: bench steps of cfg2 and cfg3 with the round's earlier sort (count/scan/place,
# Hillis-Steele scans; ab/base) against the two-launch sort (ab/new), interleaved on one box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_order_ab
mkdir -p $O
for i in 1 2 3; do
  for b in base new; do
    MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/$b/libmsv_hip.so timeout -k 10 240 python bench.py --config cfg2 --no-cpu --steps 100 > $O/cfg2_${b}_$i.json 2> $O/cfg2_${b}_$i.err
  done
done
for i in 1 2; do
  for b in base new; do
    MSV_LIB_PATH=$GRAFT_REPO_ROOT/ab/$b/libmsv_hip.so timeout -k 10 240 python bench.py --config cfg3 --no-cpu --steps 40 > $O/cfg3_${b}_$i.json 2> $O/cfg3_${b}_$i.err
  done
done
