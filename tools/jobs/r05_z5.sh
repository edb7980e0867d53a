# Round 5 job Z5: workgroups of the single-wave Viterbi kernel that have no sequence leave before staging
# their tables (early) vs HEAD, on cfg2 in place; then the GPU suite, smoke and bench cfg2 / cfg3 at the new
# in-tree build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z5
mkdir -p $O
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s2_t7 --rounds 3 abx/tbase/libmsv_hip.so abx/early/libmsv_hip.so > $O/ab_vit_cfg2.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 150 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
