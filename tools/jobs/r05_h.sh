# Round 5 job H: team variants with phase-A (and DM) transitions in LDS -- three waves per SIMD for the
# two-wave teams -- parity, then timing against the current picks on cfg5 survivors and the bands.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --longest-first --rounds 2 --variants vit_w2_s19_g,vit_w2_s19_gb > $O/tune_cfg5.jsonl
T="timeout -k 10 150 python tools/vit_tune.py --n 7000 --lmin 300 --lmax 500 --rounds 2"
$T --profile 1509.hmm --variants vit_w2_s12_g,vit_w2_s12_ga > $O/tune_bands.jsonl
$T --profile 1901.hmm --variants vit_s30_t0g,vit_w2_s15_g,vit_w2_s15_ga >> $O/tune_bands.jsonl
$T --profile 2138.hmm --variants vit_w2_s17_g,vit_w2_s17_gb >> $O/tune_bands.jsonl
$T --profile 2207.hmm --variants vit_w2_s18_g,vit_w2_s18_gb >> $O/tune_bands.jsonl
$T --profile 1600.hmm --variants vit_s26_t0g,vit_w2_s13_e >> $O/tune_bands.jsonl
