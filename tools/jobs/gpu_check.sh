# GPU parity suite, then the cfg5 bench line (BIG profile).
set -e
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --config cfg5 --steps 5 --warmup 2 > gpurun_out/bench_cfg5.log 2>&1
