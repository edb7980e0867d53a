# 4-lane throughput plan for the smallest profiles: GPU suite, smoke, bench cfg2, sweeps at 100k / 30k / 10k.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_narrow
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
for n in 100000 30000 10000; do
timeout -k 10 300 python tools/profile_sweep.py --config cfg3 --n $n --time 20 >> $O/sweep.jsonl
done
