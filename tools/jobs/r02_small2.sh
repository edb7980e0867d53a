# Small profiles: 4/8-lane throughput variants against the 16-lane ones by batch size (crossover).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_small
mkdir -p $O
for n in 10000 20000 30000 50000 70000; do
  echo "{\"profile\": \"100.hmm\", \"n\": $n}" >> $O/tune_small2.jsonl
  timeout -k 10 300 python tools/tune.py --profile 100.hmm --n $n --rounds 2 --variants msv_g16_s8_w4_p2_d1,msv_g4_s28_w8_p7_d1,msv_g4_s28_w16_p7_d1,msv_g8_s16_w8_p4_d1 >> $O/tune_small2.jsonl
done
for n in 10000 30000 50000 100000; do
  echo "{\"profile\": \"200.hmm\", \"n\": $n}" >> $O/tune_small2.jsonl
  timeout -k 10 300 python tools/tune.py --profile 200.hmm --n $n --rounds 2 --variants msv_g16_s16_w8_p2_d1,msv_g16_s16_w16_p4_d1,msv_g8_s32_w16_p8_d1 >> $O/tune_small2.jsonl
done
