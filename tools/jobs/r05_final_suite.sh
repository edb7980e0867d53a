# Round 5: the GPU suite and smoke at the very last HEAD (the bench kernels' ISA is the closing pass's,
# tools/jobs/r05_final.sh -> gpurun_out/r05_final2; this HEAD adds the inline fix for S = 14..24 and the
# scratch test), then the cfg3 bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_final_suite
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
