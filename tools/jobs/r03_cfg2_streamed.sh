# cfg2's streamed host path (msv_score_batch_async, two calls in flight): re-measure, and trace the calls.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_cfg2_streamed
mkdir -p $O
timeout -k 10 300 python bench.py --config cfg2 --no-cpu > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --config cfg2 --calls 5 --mark 2 --streamed 12 > $O/trace.out 2> $O/trace.err
python3 tools/pipeline_timeline.py $(find $O/trace -name '*kernel_trace.csv') $(find $O/trace -name '*memory_copy_trace.csv') > $O/timeline.txt 2>&1
