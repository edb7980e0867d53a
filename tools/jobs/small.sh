set -e
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 200 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1 --rounds 2 --reps 5 > gpurun_out/tune_100.log 2>&1
timeout -k 10 200 python tools/tune.py --profile 400.hmm --n 10000 --lmin 300 --lmax 500 --seed 1 --rounds 1 --reps 5 > gpurun_out/tune_400.log 2>&1
timeout -k 10 200 python tools/tune.py --profile 1400.hmm --n 100000 --lmin 300 --lmax 500 --seed 2 --rounds 1 --reps 3 --variants msv_g16_s88_w16_p2_d1 > gpurun_out/tune_1400.log 2>&1
