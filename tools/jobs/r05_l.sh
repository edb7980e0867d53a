# Round 5 closing job: GPU suite + smoke at HEAD, bench lines cfg3 / cfg5 / cfg2 / cfg4 (the Viterbi stage's
# team picks in cfg5's line), rocprofv3 kernel-trace summaries + exact-variant windows of the cfg3 and cfg5
# bench commands.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 200 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 150 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
for c in cfg3 cfg5; do
  case $c in cfg5) ST=10;; *) ST=20;; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python3 bench.py --config $c --no-cpu --no-clock --steps $ST > $O/bench_${c}_rocprof.json 2> $O/bench_${c}_rocprof.err
  V=$(python3 -c "import json;print(json.load(open('$O/bench_${c}_rocprof.json'))['config']['kernel_variant'])")
  python3 tools/rocprof_window.py $(find $O/trace_$c -name '*kernel_trace.csv') --variant $V --last $ST > $O/window_$c.json
  cp $(find $O/trace_$c -name '*kernel_stats.csv') $O/kernel_stats_$c.csv
  rm -rf $O/trace_$c
done
timeout -k 10 250 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
