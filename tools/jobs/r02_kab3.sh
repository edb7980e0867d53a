set -e
O=gpurun_out/r02_kab3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --config cfg2 --no-cpu > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3_q8.json 2> $O/bench_cfg3_q8.err
