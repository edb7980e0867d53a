# Kernel timing through launch-updated events: bench lines cfg2/cfg3 + rocprof window of cfg3 (agreement).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M=gpurun_out/r02_ev
mkdir -p $M
timeout -k 10 300 python bench.py --config cfg2 --no-cpu > $M/bench_cfg2.json 2> $M/bench_cfg2.err
timeout -k 10 300 python bench.py --no-cpu > $M/bench_cfg3.json 2> $M/bench_cfg3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench -o run -- python3 bench.py --no-cpu > $M/bench_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench/run_kernel_trace.csv --last 20 > $M/rocprof_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_cfg2 -o run -- python3 bench.py --no-cpu --config cfg2 > $M/bench_cfg2_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_cfg2/run_kernel_trace.csv --last 20 > $M/rocprof_window_cfg2.json
