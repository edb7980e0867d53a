set -e
timeout -k 10 200 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1 --rounds 2 --reps 5 --variants msv_g16_s8_w4_p2_d1,exp32_g16_s8_w4_p2_d1,msv_g16_s8_w16_p2_d1,exp32_g16_s8_w16_p2_d1 > gpurun_out/tune_exp32.log 2>&1
timeout -k 10 200 python tools/tune.py --profile 1400.hmm --n 100000 --lmin 300 --lmax 500 --seed 2 --rounds 1 --reps 3 --variants msv_g16_s88_w16_p2_d1,exp32_g16_s88_w16_p2_d1 >> gpurun_out/tune_exp32.log 2>&1
