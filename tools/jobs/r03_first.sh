# Round-3 first GPU pass: parity suite (new: full-size cfg2/cfg3 vs oracle, bad order entries), bench
# cfg3 (driver shape), the 2-rank launcher rehearsal, cfg4 rocprofv3 kernel trace + exact-variant
# window, cfg2 PMC through the name-checked summary.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_first
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
MSV_BENCH_BACKEND=gloo MSV_BENCH_ONE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --config cfg4 --steps 3 --warmup 1 --no-cpu > $O/rehearse_cfg4_2rank.json 2> $O/rehearse_cfg4_2rank.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg4_trace -o run -- python3 bench.py --config cfg4 --no-cpu --steps 10 --warmup 5 > $O/bench_cfg4_rocprof.json 2> $O/bench_cfg4_rocprof.err
T=$(find $O/cfg4_trace -name '*kernel_trace.csv')
cp $(find $O/cfg4_trace -name '*kernel_stats.csv') $O/cfg4_kernel_stats.csv
python3 tools/rocprof_window.py $T --variant $(python3 -c "import json;print(json.load(open('$O/bench_cfg4_rocprof.json'))['config']['kernel_variant'])") --last 10 > $O/cfg4_window.json
bash tools/pmc.sh cfg2 $O/pmc_cfg2 > $O/pmc_cfg2.log 2>&1
