# rocprofv3 kernel stats + timed window of the cfg3 and cfg5 bench commands (bench's timed steps are the
# last MSV dispatches again), and the cfg3 bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M=gpurun_out/prof3
mkdir -p $M
timeout -k 10 300 python bench.py > $M/bench_cfg3.json 2> $M/bench_cfg3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench -o run -- python3 bench.py --no-cpu > $M/bench_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench/run_kernel_trace.csv --last 20 > $M/rocprof_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench_cfg5 -o run -- python3 bench.py --no-cpu --config cfg5 --steps 5 > $M/bench_cfg5_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench_cfg5/run_kernel_trace.csv --last 5 > $M/rocprof_window_cfg5.json
