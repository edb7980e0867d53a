set -e
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
for p in 1901 2050 2207 2365; do
  timeout -k 10 200 python tools/tune.py --profile $p.hmm --n 10000 --lmin 1500 --lmax 2500 --seed 4 --rounds 1 --reps 2 > gpurun_out/tune_$p.log 2>&1
done
