# The split cooperative plan (1465-2480 states): GPU suite, then the reference's benchmark programs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_coop_split
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_reference_programs.py > $O/reference_programs.json 2> $O/reference_programs.err
