# Async host batches with the offsets' H2D on a stream of its own (the copy stream carries only residues;
# the order starts once the offsets land): async/pinned tests, cfg2/cfg3 bench lines (streamed fraction),
# cfg2 streamed timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_async_offsets
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "async or pinned or zero_copy or stream" > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --config cfg2 --calls 5 --mark 1 --streamed 30 > $O/calls.txt 2> $O/calls.err
python3 tools/pipeline_timeline.py $(find $O/trace -name '*kernel_trace.csv') $(find $O/trace -name '*memory_copy_trace.csv') > $O/timeline.txt 2>&1
