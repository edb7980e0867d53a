# Mid plan candidates for 600-900-state profiles (main S = 40-60): latency / 32-lane / 16-lane plans forced.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_mid3
mkdir -p $O
run() {  # profile variants
  for n in 6000 9000 12000 16000 24000; do
    echo "{\"profile\": \"$1\", \"n\": $n}" >> $O/tune_mid3.jsonl
    timeout -k 10 200 python tools/tune.py --profile $1 --n $n --rounds 2 --variants $2 >> $O/tune_mid3.jsonl
  done
}
run 600.hmm msv_g64_s12_w16_p3_d1,msv_g32_s20_w12_p2_d1,msv_g16_s40_w8_p2_d1
run 800.hmm msv_g64_s16_w16_p4_d1,msv_g32_s28_w16_p2_d1,msv_g16_s52_w12_p2_d1
run 900.hmm msv_g64_s16_w16_p4_d1,msv_g32_s32_w16_p2_d1,msv_g16_s60_w8_p2_d1
