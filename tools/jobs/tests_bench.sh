# pytest -m gpu, then the default bench line without the CPU baseline (quick check).
set -e
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_cfg3.json 2>/dev/null
