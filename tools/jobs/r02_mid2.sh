# Mid-size batches: latency (G = 64) vs mid (G = 32) vs main (G = 16) plans over profile sizes and batch sizes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_mid
mkdir -p $O
run() {  # profile variants
  for n in 3000 6000 9000 12000 16000 24000 32000; do
    echo "{\"profile\": \"$1\", \"n\": $n}" >> $O/tune_mid.jsonl
    timeout -k 10 200 python tools/tune.py --profile $1 --n $n --rounds 2 --variants $2 >> $O/tune_mid.jsonl
  done
}
run 500.hmm msv_g64_s8_w16_p2_d1,msv_g32_s16_w12_p2_d1,msv_g16_s32_w12_p2_d1
run 700.hmm msv_g64_s12_w16_p3_d1,msv_g32_s24_w16_p2_d1,msv_g16_s44_w12_p2_d1
run 1001.hmm msv_g64_s16_w16_p4_d1,msv_g32_s32_w16_p2_d1,msv_g16_s64_w16_p2_d1
run 1200.hmm msv_g64_s20_w16_p5_d1,msv_g32_s40_w16_p2_d1,msv_g16_s76_w16_p2_d1
run 1400.hmm msv_g64_s24_w16_p6_d1,msv_g32_s44_w16_p2_d1,msv_g16_s88_w16_p2_d1
run 1509.hmm msv_g64_s24_w16_p6_d1,msv_g32_s48_w16_p2_d1,msv_g16_s96_w12_p2_d1
