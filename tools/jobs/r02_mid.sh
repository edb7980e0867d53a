# Mid-size batches (between the latency plan's limit and one round of the main grid): 1400.hmm and
# 1001.hmm, latency (G = 64), main (G = 16) and G = 32 variants at 6k..48k sequences.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_mid
mkdir -p $O
for n in 6000 10000 14000 20000 32000 48000; do
timeout -k 10 200 python tools/tune.py --profile 1400.hmm --n $n --rounds 2 --variants msv_g64_s24_w16_p6_d1,msv_g16_s88_w16_p2_d1,msv_g32_s44_w16_p2_d1,msv_g32_s44_w12_p2_d2 >> $O/tune_1400.jsonl
done
for n in 6000 10000 16000 24000; do
timeout -k 10 200 python tools/tune.py --profile 1001.hmm --n $n --rounds 2 --variants msv_g64_s16_w16_p4_d1,msv_g16_s64_w16_p2_d1 >> $O/tune_1001.jsonl
done
