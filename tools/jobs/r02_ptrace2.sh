# Host pipeline timeline (one call + a stream of async calls on two compute streams), cfg3 bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_ptrace2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --streamed 10 > $O/calls.log 2>&1
python3 tools/pipeline_timeline.py $O/trace/run_kernel_trace.csv $O/trace/run_memory_copy_trace.csv > $O/timeline.txt
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
