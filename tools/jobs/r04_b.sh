# Round 4 job B: the whole GPU suite at this HEAD (cfg4/cfg5 every score, grid ADVICE fixes, Viterbi),
# smoke, then bench cfg3 (Viterbi-stage figure, clock twin) and cfg2.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 200 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
