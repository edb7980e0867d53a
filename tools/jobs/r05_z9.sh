# Round 5 job Z9: short Viterbi rows (S < 8): the first lazy-F passes over whole-lane hops unconditionally
# (8 or 16 states' worth) vs ballot-first (h0) -- cfg2 in place (100.hmm, S = 2), 200.hmm / 300.hmm random
# batches small (latency-bound) and large; the Viterbi tests on h8.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z9
mkdir -p $O
MSV_LIB_PATH=$PWD/abx/h8/libmsv_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests_h8.txt 2>&1
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s2_t7 --rounds 3 abx/h0/libmsv_hip.so abx/h8/libmsv_hip.so abx/h16/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 300 --profile 200.hmm --variant vit_s4_t7 --rounds 2 abx/h0/libmsv_hip.so abx/h8/libmsv_hip.so abx/h16/libmsv_hip.so > $O/ab_200_n300.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 200.hmm --variant vit_s4_t7 --rounds 2 abx/h0/libmsv_hip.so abx/h8/libmsv_hip.so abx/h16/libmsv_hip.so > $O/ab_200_n20000.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 20000 --profile 100.hmm --variant vit_s2_t7 --rounds 2 abx/h0/libmsv_hip.so abx/h8/libmsv_hip.so abx/h16/libmsv_hip.so > $O/ab_100_n20000.jsonl
