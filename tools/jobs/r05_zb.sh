# Round 5 job ZB: the single-wave Viterbi kernel's short rows (S <= 8, transitions in VGPRs) with the next
# row's match scores requested during the row (XROW) vs HEAD: cfg2 in place, 200.hmm x 300 (latency-bound),
# 100 / 200 / 500.hmm x 20k (throughput); the Viterbi tests on the new in-tree build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s2_t7 --rounds 3 abx/base/libmsv_hip.so abx/xrow/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 300 --profile 200.hmm --variant vit_s4_t7 --rounds 2 abx/base/libmsv_hip.so abx/xrow/libmsv_hip.so > $O/ab_200_n300.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 100.hmm --variant vit_s2_t7 --rounds 2 abx/base/libmsv_hip.so abx/xrow/libmsv_hip.so > $O/ab_100_n20000.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 200.hmm --variant vit_s4_t7 --rounds 2 abx/base/libmsv_hip.so abx/xrow/libmsv_hip.so > $O/ab_200_n20000.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 500.hmm --variant vit_s8_t7 --rounds 2 abx/base/libmsv_hip.so abx/xrow/libmsv_hip.so > $O/ab_500_n20000.jsonl
