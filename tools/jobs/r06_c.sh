# Round 6: interleaved A/Bs of the W = 2 team exchange with per-half stamps, second form (wave 0 writes {E, M}
# when its row ends and {I, D} after its lazy-F; wave 1 spins on {I, D} alone, then reads {E, M}): HEAD~ before the
# exchange change (r6base) vs it (r6x5) on cfg5's survivors (w2_s19_gb), cfg3's (w1_s22_ea, no exchange), and
# 7,000-sequence bands of 1600.hmm (w2_s13_ga4: 14 -> 39 spilled VGPRs), 1509.hmm (w2_s12_ga4), 2207.hmm (w2_s18_gb).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_c
mkdir -p $O
timeout -k 10 240 python -u tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 3 --in-place abx/r6base/libmsv_hip.so abx/r6x5/libmsv_hip.so > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1600.hmm --variant vit_w2_s13_ga4 --rounds 3 abx/r6base/libmsv_hip.so abx/r6x5/libmsv_hip.so > $O/ab_1600.jsonl 2> $O/ab_1600.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1509.hmm --variant vit_w2_s12_ga4 --rounds 3 abx/r6base/libmsv_hip.so abx/r6x5/libmsv_hip.so > $O/ab_1509.jsonl 2> $O/ab_1509.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 2207.hmm --variant vit_w2_s18_gb --rounds 3 abx/r6base/libmsv_hip.so abx/r6x5/libmsv_hip.so > $O/ab_2207.jsonl 2> $O/ab_2207.err
timeout -k 10 150 python -u tools/vit_ab.py --config cfg3 --variant vit_w1_s22_ea --rounds 2 --in-place abx/r6base/libmsv_hip.so abx/r6x5/libmsv_hip.so > $O/ab_cfg3.jsonl 2> $O/ab_cfg3.err
