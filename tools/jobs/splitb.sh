# Split layout (2405.hmm, cfg5 shape): the cost of the B-block L2 reads (EXP & 65536: B halves from
# LDS, wrong scores) and of their VMEM issue count (EXP & 131072: float4 instead of float2 loads,
# wrong scores), against the production variant, interleaved in one process:
#   EXPERIMENTS=1 bash tools/ab_build.sh . exp;  gpurun -- 'bash tools/jobs/splitb.sh'
set -e
O=gpurun_out/splitb
mkdir -p $O
MSV_LIB_PATH=$PWD/ab/exp/libmsv_hip.so timeout -k 10 300 python tools/tune.py --profile 2405.hmm --n 100000 --lmin 1500 \
  --lmax 2500 --seed 4000 --rounds 2 --reps 3 \
  --variants msv_g32_s76_a64_w16_p2_d1,exp65536_g32_s76_a64_w16_p2_d1,exp131072_g32_s76_a64_w16_p2_d1 \
  > $O/tune_2405.jsonl 2> $O/tune_2405.err
cat $O/tune_2405.jsonl
