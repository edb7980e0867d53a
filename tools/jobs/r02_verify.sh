# Round-2 re-entry check of HEAD: GPU parity suite, smoke, default bench (cfg3) and its rocprofv3 stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_verify
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu > $O/bench_cfg3_prof.json 2> $O/bench_cfg3_prof.err
