# Round-2 measurement pass at HEAD (zero-copy host path, small-batch assignment, latency plans): bench lines cfg3/cfg2/
# cfg5/cfg4, rocprofv3 kernel stats + timed window of the cfg3 and cfg5 bench commands, PMC for cfg3
# and cfg2, cfg2 without the longest-first order, the cfg5 wave timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
M=gpurun_out/measure3
mkdir -p $M
timeout -k 10 300 python bench.py > $M/bench_cfg3.json 2> $M/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg2 > $M/bench_cfg2.json 2> $M/bench_cfg2.err
timeout -k 10 300 python tools/bench_reference_programs.py > $M/refprog.json 2> $M/refprog.err
timeout -k 10 300 python bench.py --config cfg5 --steps 5 > $M/bench_cfg5.json 2> $M/bench_cfg5.err
timeout -k 10 400 python bench.py --config cfg4 --steps 10 > $M/bench_cfg4.json 2> $M/bench_cfg4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench -o run -- python3 bench.py --no-cpu > $M/bench_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench/run_kernel_trace.csv --last 20 > $M/rocprof_window.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $M/rocprof_bench_cfg5 -o run -- python3 bench.py --no-cpu --config cfg5 --steps 5 > $M/bench_cfg5_under_rocprof.json 2>&1
python3 tools/rocprof_window.py $M/rocprof_bench_cfg5/run_kernel_trace.csv --last 5 > $M/rocprof_window_cfg5.json
timeout -k 10 200 python tools/wave_timeline.py --config cfg5 > $M/timeline_cfg5.jsonl
timeout -k 10 200 python tools/wave_timeline.py --config cfg3 >> $M/timeline_cfg3.jsonl
timeout -k 10 900 bash tools/pmc.sh cfg3 $M/pmc_cfg3 > $M/pmc_cfg3.log 2>&1
timeout -k 10 900 bash tools/pmc.sh cfg2 $M/pmc_cfg2 > $M/pmc_cfg2.log 2>&1
