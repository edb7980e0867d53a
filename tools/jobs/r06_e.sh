# Round 6: the W = 2 team exchange's torn-safe forms, interleaved vs HEAD (r6base): r6x8 = round 5's protocol
# with {E_0, st, I, st} / {M, st, D, st} records, each spin on ONE stamp word then the other checked once;
# r6x9 = r6x8 + s_sleep 1 after a failed poll; r6x7 = every stamp checked per try + s_sleep 1.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_e
mkdir -p $O
L="abx/r6base/libmsv_hip.so abx/r6x8/libmsv_hip.so abx/r6x9/libmsv_hip.so abx/r6x7/libmsv_hip.so"
timeout -k 10 300 python -u tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 2 --in-place $L > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1600.hmm --variant vit_w2_s13_ga4 --rounds 2 $L > $O/ab_1600.jsonl 2> $O/ab_1600.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 2207.hmm --variant vit_w2_s18_gb --rounds 2 $L > $O/ab_2207.jsonl 2> $O/ab_2207.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1509.hmm --variant vit_w2_s12_ga4 --rounds 2 $L > $O/ab_1509.jsonl 2> $O/ab_1509.err
