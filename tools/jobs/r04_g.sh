# Round 4 job G: Viterbi GPU tests and the per-S variant choice: interleaved timings of the candidate forms
# on the cfg3 survivors (longest first, as the pipeline lists them) and on random batches of the profiles
# whose model lengths need S = 20, 24, 26, 30, 34, 36.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
T="timeout -k 10 200 python tools/vit_tune.py --rounds 3"
$T --config cfg3 --longest-first --variants vit_s22_t5a,vit_s22_t5,vit_s22_t0w12,vit_s22_t0w12a,vit_s24_t7w4,vit_s24_t0g > $O/tune_cfg3.jsonl 2> $O/tune.err
$T --profile 1200.hmm --n 7000 --variants vit_s20_t5a,vit_s20_t5,vit_s22_t5a,vit_s24_t0g > $O/tune_1200.jsonl 2>> $O/tune.err
$T --profile 1509.hmm --n 7000 --variants vit_s24_t7w4,vit_s24_t0g,vit_s24_t5,vit_s26_t0g,vit_s28_t0g > $O/tune_1509.jsonl 2>> $O/tune.err
$T --profile 1600.hmm --n 7000 --variants vit_s26_t0g,vit_s26_t7w4,vit_s28_t0g,vit_s28_t7w4 > $O/tune_1600.jsonl 2>> $O/tune.err
$T --profile 1901.hmm --n 7000 --variants vit_s30_t0g,vit_s32_t0g,vit_s34_t7gw4 > $O/tune_1901.jsonl 2>> $O/tune.err
$T --profile 2138.hmm --n 7000 --variants vit_s34_t7gw4,vit_s36_t7gw4,vit_s38_t7gw4,vit_s38_t0g4 > $O/tune_2138.jsonl 2>> $O/tune.err
