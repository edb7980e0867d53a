set -e
timeout -k 10 400 python tools/tune.py --profile 2405.hmm --n 20000 --lmin 1500 --lmax 2500 --seed 4 --rounds 3 --reps 2 --variants msv_g64_s40_w16_p2_d1,exp4096_g64_s40_w16_p2_d1 > gpurun_out/ab_big.log 2>&1
timeout -k 10 420 python -m pytest tests -m gpu -x -q -k "variant or 2405 or latency or synthetic" > gpurun_out/pytest_gpu.log 2>&1
