# Host paths with kernel-written pinned destinations, async calls on two compute streams, sorts without
# a memset: GPU suite, pipeline timeline, cfg3 bench line (end_to_end), cfg3 kernel A/B vs ab/first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_host2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --streamed 10 > $O/calls.log 2>&1
python3 tools/pipeline_timeline.py $O/trace/run_kernel_trace.csv $O/trace/run_memory_copy_trace.csv > $O/timeline.txt
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --no-cpu --config cfg4 --steps 5 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
