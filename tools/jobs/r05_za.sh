# Round 5 job ZA: the short-row hops chosen at run time per launch (latency-bound: total <= grid waves; the row loop
# compiled twice, the branch outside it) vs HEAD -- cfg2 in place, 200.hmm x 300, and the throughput shapes 100 / 200.hmm x 20k; Viterbi tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_za2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s2_t7 --rounds 3 abx/base/libmsv_hip.so abx/few2/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 300 --profile 200.hmm --variant vit_s4_t7 --rounds 2 abx/base/libmsv_hip.so abx/few2/libmsv_hip.so > $O/ab_200_n300.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 200.hmm --variant vit_s4_t7 --rounds 2 abx/base/libmsv_hip.so abx/few2/libmsv_hip.so > $O/ab_200_n20000.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 100.hmm --variant vit_s2_t7 --rounds 2 abx/base/libmsv_hip.so abx/few2/libmsv_hip.so > $O/ab_100_n20000.jsonl
