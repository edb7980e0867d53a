# Full measurement pass for one round: bench lines (cfg3 default + cfg2/cfg5), the rocprofv3
# kernel-trace/stats summary of the default bench command, and the PMC passes for cfg3.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/measure
timeout -k 10 300 python bench.py > gpurun_out/measure/bench_cfg3.json 2> gpurun_out/measure/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg2 > gpurun_out/measure/bench_cfg2.json 2> gpurun_out/measure/bench_cfg2.err
timeout -k 10 300 python bench.py --config cfg5 --steps 5 > gpurun_out/measure/bench_cfg5.json 2> gpurun_out/measure/bench_cfg5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/measure/rocprof_bench -o run -- python3 bench.py --no-cpu > gpurun_out/measure/bench_under_rocprof.json 2>&1
python3 tools/rocprof_window.py gpurun_out/measure/rocprof_bench/run_kernel_trace.csv --skip 12 --take 20 > gpurun_out/measure/rocprof_window.json
timeout -k 10 900 bash tools/pmc.sh cfg3 gpurun_out/measure/pmc_cfg3 > gpurun_out/measure/pmc.log 2>&1
