# Round 5 job Z2: the Viterbi stage on cfg2's 260 survivors (latency-bound: one wave per sequence, at most
# one per SIMD) -- the single-wave picks vs W = 1 team variants with the phase-A/B row; Viterbi tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k "every_variant or team" --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg2 --in-place --rounds 3 --variants vit_s2_t7,vit_s4_t7,vit_w1_s2_e,vit_w1_s3_e,vit_w1_s4_e,vit_w1_s8_e > $O/tune_cfg2.jsonl
timeout -k 10 300 python tools/vit_tune.py --profile 100.hmm --n 2000 --rounds 3 --variants vit_s2_t7,vit_w1_s2_e,vit_w1_s4_e > $O/tune_100_n2000.jsonl
timeout -k 10 300 python tools/vit_tune.py --profile 200.hmm --n 1000 --rounds 3 --variants vit_s4_t7,vit_w1_s4_e,vit_w1_s8_e > $O/tune_200_n1000.jsonl
