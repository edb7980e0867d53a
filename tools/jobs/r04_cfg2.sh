# Round 4, cfg2: the measured floor of the g16_s8 row chain, then A/B of two sequences
# per lane group (D = 2) and 8 lanes x 16 states against the production plan at n = 10k (bitwise-checked
# by tune.py across the variants).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_cfg2
mkdir -p $O
timeout -k 10 240 python tools/cfg2_floor.py --out $O/cfg2_floor.json > $O/cfg2_floor.log 2>&1
timeout -k 10 400 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1000 --rounds 4 \
  --variants msv_g16_s8_w4_p2_d1,msv_g16_s8_w4_p2_d2,msv_g16_s8_w8_p2_d2,msv_g8_s16_w16_p4_d1,msv_g8_s16_w8_p4_d1,msv_g16_s8_w8_p2_d1 \
  > $O/tune_cfg2.jsonl 2> $O/tune_cfg2.err
