set -e
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python tools/tune.py --profile 1400.hmm --n 100000 --lmin 300 --lmax 500 --seed 2 --rounds 3 --reps 3 --variants msv_g16_s88_w16_p2_d1,exp2048_g16_s88_w16_p2_d1 > gpurun_out/ab.log 2>&1
timeout -k 10 400 python tools/tune.py --profile 2405.hmm --n 20000 --lmin 1500 --lmax 2500 --seed 4 --rounds 2 --reps 2 --variants msv_g64_s40_w16_p2_d1,exp2048_g64_s40_w16_p2_d1 > gpurun_out/ab_big.log 2>&1
timeout -k 10 400 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1 --rounds 3 --reps 5 --variants msv_g16_s8_w4_p2_d1,exp2048_g16_s8_w4_p2_d1 > gpurun_out/ab_small.log 2>&1
