# PMC passes at HEAD for cfg2/3/4/5 (tools/pmc.sh: name-checked, calibrated summaries).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_pmc_head
mkdir -p $O
for c in cfg2 cfg3 cfg5 cfg4; do
  timeout -k 10 600 bash tools/pmc.sh $c $O/pmc_$c > $O/pmc_$c.log 2>&1
done
