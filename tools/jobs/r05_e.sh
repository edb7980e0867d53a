# Round 5 job E: team variants (vit_team.hip) against the single-wave picks per profile band (random
# 7,000 x U[300,500] batches, as profiles/r04_vit_tune_picks.jsonl) and on the cfg5 survivors; parity of
# the new team shapes first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 120 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
T="timeout -k 10 150 python tools/vit_tune.py --n 7000 --lmin 300 --lmax 500 --rounds 2"
$T --profile 1509.hmm --variants vit_s24_t0g,vit_w2_s12_e,vit_w2_s12_g > $O/tune_bands.jsonl
$T --profile 1600.hmm --variants vit_s26_t0g,vit_w2_s13_e,vit_w2_s13_g >> $O/tune_bands.jsonl
$T --profile 1705.hmm --variants vit_s28_t0g,vit_w2_s14_e,vit_w2_s14_g >> $O/tune_bands.jsonl
$T --profile 1901.hmm --variants vit_s30_t0g,vit_w2_s15_g >> $O/tune_bands.jsonl
$T --profile 2050.hmm --variants vit_s34_t7gw4,vit_w2_s17_g >> $O/tune_bands.jsonl
$T --profile 2138.hmm --variants vit_s34_t7gw4,vit_w2_s17_g >> $O/tune_bands.jsonl
$T --profile 2207.hmm --variants vit_s36_t7gw4,vit_w2_s18_g >> $O/tune_bands.jsonl
$T --profile 2365.hmm --variants vit_s38_t7gw4,vit_w2_s19_g >> $O/tune_bands.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --longest-first --rounds 2 --variants vit_s38_t7gw4,vit_w2_s19_g > $O/tune_cfg5.jsonl
