# Round 4 job B: Viterbi GPU tests (incl. the ascending-pass variants) and variant timing on cfg3 / cfg2 MSV
# survivors, then the whole GPU suite (cfg4/cfg5 every score, grid ADVICE fixes), smoke, bench cfg3 and cfg2.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
timeout -k 10 200 python tools/vit_tune.py --config cfg3 --rounds 3 > $O/vit_tune_cfg3.jsonl 2> $O/vit_tune_cfg3.err
timeout -k 10 150 python tools/vit_tune.py --config cfg2 --rounds 3 > $O/vit_tune_cfg2.jsonl 2> $O/vit_tune_cfg2.err
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_viterbi.py > $O/pytest_gpu.log 2>&1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
