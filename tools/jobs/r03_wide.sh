# Wide-block zero-copy twins + fused offsets copy: new parity tests, the zero-copy suite, A/B of the
# twins (64-B superblocks vs 16-B blocks) per shape, cfg2/cfg3 bench lines, cfg2 host-call timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_wide
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "zero_copy or pinned or async or cfg2" > $O/pytest_zc.log 2>&1
timeout -k 10 300 python tools/zc_wide_ab.py --rounds 3 > $O/ab.jsonl 2> $O/ab.err
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --config cfg2 --calls 30 --mark 3 > $O/calls.txt 2> $O/calls.err
python3 tools/pipeline_timeline.py $(find $O/trace -name '*kernel_trace.csv') $(find $O/trace -name '*memory_copy_trace.csv') > $O/timeline.txt 2>&1
