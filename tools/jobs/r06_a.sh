# Round 6, first GPU job: the reference's own callers built unchanged against the library (test_MSV over 24
# profiles, benchmark_MSV / benchmark_MSV_1400 outputs), then the whole GPU suite and a cfg3 bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_a
mkdir -p $O/callers
REF_CALLERS_OUT=$O/callers timeout -k 10 300 python -u -m pytest tests/test_ref_callers.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/ref_callers.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
