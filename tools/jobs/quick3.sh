# pytest -m gpu, then bench lines for cfg3 / cfg2 / cfg5 without the CPU baseline (A/B check).
set -e
mkdir -p gpurun_out/quick3
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick3/pytest_gpu.log 2>&1
for c in cfg3 cfg2 cfg5; do
  timeout -k 10 300 python bench.py --no-cpu --config $c > gpurun_out/quick3/bench_$c.json 2> gpurun_out/quick3/bench_$c.err
done
