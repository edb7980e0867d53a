# Round 5 job U: drain-tail fairness A/B (VIT_TAIL_PRIO: issue priority from the remaining rows) on the S = 22
# pick: cfg3's survivors, 3,072 equal-length sequences (one per wave) and 7,261 random U[300, 500].
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_u
mkdir -p $O
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --variant vit_w1_s22_ea --rounds 3 abx/tbase/libmsv_hip.so abx/tprio/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 3072 --lmin 400 --lmax 400 --variant vit_w1_s22_ea --rounds 2 abx/tbase/libmsv_hip.so abx/tprio/libmsv_hip.so > $O/ab_n3072.jsonl
timeout -k 10 300 python tools/vit_ab.py --n 7261 --variant vit_w1_s22_ea --rounds 2 abx/tbase/libmsv_hip.so abx/tprio/libmsv_hip.so > $O/ab_n7261.jsonl
