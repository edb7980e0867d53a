# Host pipeline: new GPU tests (async, pieces), piece-plan sweep, cfg3 bench line.
set -e
O=gpurun_out/r02_pipe
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_configs.log 2>&1
timeout -k 10 300 python tools/host_pipeline_sweep.py --config cfg3 > $O/sweep_cfg3.jsonl 2> $O/sweep_cfg3.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
