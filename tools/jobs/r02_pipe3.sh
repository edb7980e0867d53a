set -e
O=gpurun_out/r02_pipe3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_configs.log 2>&1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/host_pipeline_sweep.py --config cfg3 > $O/sweep_cfg3.jsonl 2> $O/sweep_cfg3.err
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --no-cpu --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
