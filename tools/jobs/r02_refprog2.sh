# Grid fixes (largest first, errors from scores): parity tests + reference programs at 8 HW queues.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_refprog2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_reference_programs.py > $O/refprog.json 2> $O/refprog.err
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python tools/bench_reference_programs.py > $O/refprog_q4.json 2> $O/refprog_q4.err
