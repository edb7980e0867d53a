# Round 4 closing measurements: bench lines for cfg3 (the driver's default command, CPU baseline, Viterbi
# stage, clock), cfg2, cfg5, cfg4; rocprofv3 kernel-trace summaries + exact-variant windows of the bench
# commands (the Viterbi stage's kernel is in the same traces).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_h
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 400 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
for c in cfg3 cfg2 cfg5; do
  case $c in cfg5) ST=10;; cfg2) ST=100;; *) ST=20;; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python3 bench.py --config $c --no-cpu --no-clock --steps $ST > $O/bench_${c}_rocprof.json 2> $O/bench_${c}_rocprof.err
  V=$(python3 -c "import json;print(json.load(open('$O/bench_${c}_rocprof.json'))['config']['kernel_variant'])")
  python3 tools/rocprof_window.py $(find $O/trace_$c -name '*kernel_trace.csv') --variant $V --last $ST > $O/window_$c.json
  cp $(find $O/trace_$c -name '*kernel_stats.csv') $O/kernel_stats_$c.csv
  rm -rf $O/trace_$c
done
