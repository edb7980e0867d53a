set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_pipe4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_configs.log 2>&1
timeout -k 10 300 python tools/host_pipeline_sweep.py --config cfg3 > $O/sweep_cfg3.jsonl 2> $O/sweep_cfg3.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py > $O/calls.log 2>&1
python3 tools/pipeline_timeline.py $O/trace/run_kernel_trace.csv $O/trace/run_memory_copy_trace.csv > $O/timeline.txt
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
