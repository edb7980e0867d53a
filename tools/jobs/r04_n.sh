# Round 4 job N (closing, after the Viterbi lazy-F / uniform-J changes): GPU suite + smoke, bench lines
# cfg3 / cfg2 / cfg5 / cfg4, rocprofv3 kernel-trace summary + window of the cfg3 bench command.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 400 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_cfg3 -o run -- python3 bench.py --config cfg3 --no-cpu --no-clock --steps 20 > $O/bench_cfg3_rocprof.json 2> $O/bench_cfg3_rocprof.err
python3 tools/rocprof_window.py $(find $O/trace_cfg3 -name '*kernel_trace.csv') --variant msv_g16_s88_w16_p2_d1 --last 20 > $O/window_cfg3.json
cp $(find $O/trace_cfg3 -name '*kernel_stats.csv') $O/kernel_stats_cfg3.csv
rm -rf $O/trace_cfg3
