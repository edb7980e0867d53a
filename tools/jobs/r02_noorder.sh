# cfg2 / cfg3: bench step with and without the longest-first order, interleaved (is the sort worth its
# launch for one-round batches?).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_noorder
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --config cfg2 --no-cpu --steps 50 > $O/cfg2_order_$i.json 2> $O/cfg2_order_$i.err
  timeout -k 10 240 python bench.py --config cfg2 --no-cpu --steps 50 --no-order > $O/cfg2_noorder_$i.json 2> $O/cfg2_noorder_$i.err
done
timeout -k 10 240 python bench.py --config cfg3 --no-cpu --no-order > $O/cfg3_noorder.json 2> $O/cfg3_noorder.err
