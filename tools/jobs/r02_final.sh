# Round-2 final pass at HEAD: GPU suite + smoke, bench cfg3 (default) / cfg2 / cfg4 / cfg5, rocprofv3 stats
# and timed windows of the cfg3 and cfg5 bench commands.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M=gpurun_out/final
mkdir -p $M
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $M/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $M/smoke.log 2>&1
timeout -k 10 300 python bench.py > $M/bench_cfg3.json 2> $M/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg2 > $M/bench_cfg2.json 2> $M/bench_cfg2.err
timeout -k 10 300 python bench.py --config cfg5 --steps 5 > $M/bench_cfg5.json 2> $M/bench_cfg5.err
timeout -k 10 400 python bench.py --config cfg4 --steps 10 > $M/bench_cfg4.json 2> $M/bench_cfg4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench -o run -- python3 bench.py --no-cpu > $M/bench_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench/run_kernel_trace.csv --last 20 > $M/rocprof_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench_cfg5 -o run -- python3 bench.py --no-cpu --config cfg5 --steps 5 > $M/bench_cfg5_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench_cfg5/run_kernel_trace.csv --last 5 > $M/rocprof_window_cfg5.json
