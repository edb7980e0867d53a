# Round-3 closing profile at HEAD: kernel-trace summaries + exact-variant windows of the bench commands
# (cfg2/3/4/5), PMC passes for every config through tools/pmc.sh (name-checked, calibrated).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_final_profile
mkdir -p $O
for c in cfg2 cfg3 cfg4 cfg5; do
  case $c in cfg5) ST=10;; cfg4) ST=5;; cfg2) ST=100;; *) ST=20;; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python3 bench.py --config $c --no-cpu --steps $ST > $O/bench_${c}_rocprof.json 2> $O/bench_${c}_rocprof.err
  V=$(python3 -c "import json;print(json.load(open('$O/bench_${c}_rocprof.json'))['config']['kernel_variant'])")
  python3 tools/rocprof_window.py $(find $O/trace_$c -name '*kernel_trace.csv') --variant $V --last $ST > $O/window_$c.json
  cp $(find $O/trace_$c -name '*kernel_stats.csv') $O/kernel_stats_$c.csv
done
for c in cfg2 cfg3 cfg4 cfg5; do
  bash tools/pmc.sh $c $O/pmc_$c > $O/pmc_$c.log 2>&1
done
