# Round 5 job S: the stable (order-preserving) survivor compaction: Viterbi GPU tests, in-place timing
# (bench.py's setting) of the S = 22 / 38 picks, and the cfg3 / cfg5 bench lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --in-place --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea > $O/tune_cfg3_inplace.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --in-place --rounds 2 --variants vit_s38_t7gw4,vit_w2_s19_gb > $O/tune_cfg5_inplace.jsonl
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 200 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
