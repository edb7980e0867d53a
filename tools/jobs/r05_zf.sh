# Round 5 job ZF: with two rows per trip for the LA teams, does the LA form win the S = 12 band too
# (1509.hmm: vit_w2_s12_g pick vs vit_w2_s12_ga / ga4, single-wave s24_t0g)?
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zf
mkdir -p $O
timeout -k 10 300 python tools/vit_tune.py --profile 1509.hmm --n 7000 --rounds 3 --variants vit_w2_s12_g,vit_w2_s12_ga,vit_w2_s12_ga4,vit_s24_t0g > $O/tune_1509.jsonl
timeout -k 10 300 python tools/vit_tune.py --profile 1400.hmm --n 7000 --rounds 3 --variants vit_w1_s22_ea,vit_w2_s11_ea,vit_w2_s11_ga4 > $O/tune_1400.jsonl
