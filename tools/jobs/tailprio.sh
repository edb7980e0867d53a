# Tail-priority experiment (EXP & 16384: s_setprio for the waves holding the last dequeued indices)
# against the production cfg3 variant, interleaved in one process:
#   EXPERIMENTS=1 bash tools/ab_build.sh . exp;  gpurun -- 'bash tools/jobs/tailprio.sh'
set -e
O=gpurun_out/tailprio
mkdir -p $O
MSV_LIB_PATH=$PWD/ab/exp/libmsv_hip.so timeout -k 10 300 python tools/tune.py --profile 1400.hmm --n 100000 --seed 2000 \
  --rounds 4 --reps 5 --variants msv_g16_s88_w16_p2_d1,exp16384_g16_s88_w16_p2_d1,exp49152_g16_s88_w16_p2_d1 \
  > $O/tune_1400.jsonl 2> $O/tune_1400.err
cat $O/tune_1400.jsonl
