# GPU suite after the cooperative plan's batch limit change, then the reference programs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_coop_limit
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_reference_programs.py > $O/reference_programs.json 2> $O/reference_programs.err
