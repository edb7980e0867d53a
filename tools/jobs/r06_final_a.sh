# Round 6 closing job, part A (at the final HEAD): GPU suite + smoke, bench lines cfg3 / cfg5 / cfg2 / cfg4.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_final_a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 200 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 150 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 250 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
