# Whole-row emission rings (cross-row prefetch, PF = S/4, 16 waves) against the PF-2 throughput variants
# for 200-500-state profiles at 10k and 100k sequences.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_xrow
mkdir -p $O
run() {
  for n in 10000 100000; do
    echo "{\"profile\": \"$1\", \"n\": $n}" >> $O/tune_xrow.jsonl
    timeout -k 10 200 python tools/tune.py --profile $1 --n $n --rounds 2 --variants $2 >> $O/tune_xrow.jsonl
  done
}
run 200.hmm msv_g16_s16_w8_p2_d1,msv_g16_s16_w16_p4_d1
run 300.hmm msv_g16_s20_w8_p2_d1,msv_g16_s20_w16_p5_d1
run 400.hmm msv_g16_s28_w8_p2_d1,msv_g16_s28_w16_p7_d1
run 500.hmm msv_g16_s32_w12_p2_d1,msv_g16_s32_w16_p8_d1
