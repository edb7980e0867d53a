# Round 5 job ZG: the S = 12 pick moved to vit_w2_s12_ga4 (four waves per SIMD); s13 / s14 in that form
# (14 / 20 spilled VGPRs) against their picks on 1600 / 1705.hmm; the Viterbi GPU tests (every variant).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --profile 1600.hmm --n 7000 --rounds 3 --variants vit_w2_s13_ga,vit_w2_s13_ga4 > $O/tune_1600.jsonl
timeout -k 10 300 python tools/vit_tune.py --profile 1705.hmm --n 7000 --rounds 3 --variants vit_w2_s14_ga,vit_w2_s14_ga4 > $O/tune_1705.jsonl
timeout -k 10 300 python tools/vit_tune.py --profile 1509.hmm --n 7000 --rounds 2 --variants vit_w2_s12_g,vit_w2_s12_ga4 > $O/tune_1509.jsonl
