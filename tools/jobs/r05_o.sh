# Round 5 job O: W = 1 team variants (phase-A transitions paired in LDS, three / four waves per SIMD) against
# the single-wave picks per band (random 7,000 x U[300,500]); parity of the new shapes; the 1799/1901.hmm bands.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread -k "team and w1" > $O/team_tests.txt 2>&1
T="timeout -k 10 150 python tools/vit_tune.py --n 7000 --lmin 300 --lmax 500 --rounds 2"
$T --profile 700.hmm --variants vit_s12_t7,vit_w1_s12_ea,vit_w1_s12_ea4 > $O/tune_bands.jsonl
$T --profile 800.hmm --variants vit_s14_t7,vit_w1_s14_ea,vit_w1_s14_ea4 >> $O/tune_bands.jsonl
$T --profile 1001.hmm --variants vit_s16_t7,vit_w1_s16_ea,vit_w1_s16_ea4 >> $O/tune_bands.jsonl
$T --profile 1100.hmm --variants vit_s18_t7,vit_w1_s18_ea >> $O/tune_bands.jsonl
$T --profile 1200.hmm --variants vit_s20_t5a,vit_w1_s20_ea,vit_w1_s20_eb >> $O/tune_bands.jsonl
$T --profile 1301.hmm --variants vit_s22_t5a,vit_w1_s22_ea >> $O/tune_bands.jsonl
$T --profile 1799.hmm --variants vit_s30_t0g,vit_w2_s15_ga >> $O/tune_bands.jsonl
