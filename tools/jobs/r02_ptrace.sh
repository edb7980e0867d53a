set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_ptrace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py > $O/calls.log 2>&1
python3 tools/pipeline_timeline.py $O/trace/run_kernel_trace.csv $O/trace/run_memory_copy_trace.csv > $O/timeline.txt
