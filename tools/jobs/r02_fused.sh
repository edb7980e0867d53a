# Fused grid launch (one msv_grid_kernel over all profiles for few sequences): GPU suite, reference programs
# at the default 4 and at 8 hardware queues, rocprofv3 kernel trace of the reference programs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_fused
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_reference_programs.py > $O/refprog.json 2> $O/refprog.err
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python tools/bench_reference_programs.py > $O/refprog_q4.json 2> $O/refprog_q4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o run -- python3 tools/bench_reference_programs.py > $O/refprog_rocprof.json 2>&1
timeout -k 10 300 python bench.py --config cfg2 --no-cpu > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
