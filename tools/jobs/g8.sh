# G = 8 lanes x 176 states per lane at 2 waves/SIMD (EXP & 524288: plain row_shr:1 shift, exact while
# each group's last state is padding) against the production G = 16 x 88 at 4 waves/SIMD, cfg3 shape:
#   EXPERIMENTS=1 bash tools/ab_build.sh . exp;  gpurun -- 'bash tools/jobs/g8.sh'
set -e
O=gpurun_out/g8
mkdir -p $O
MSV_LIB_PATH=$PWD/ab/exp/libmsv_hip.so timeout -k 10 300 python tools/tune.py --profile 1400.hmm --n 100000 --seed 2000 \
  --rounds 3 --reps 5 \
  --variants msv_g16_s88_w16_p2_d1,exp524288_g8_s176_w8_p2_d1,exp524288_g8_s176_w8_p3_d1,exp524288_g8_s176_w8_p4_d1 \
  > $O/tune_1400.jsonl 2> $O/tune_1400.err
cat $O/tune_1400.jsonl
