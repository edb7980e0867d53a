set -e
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_reference_programs.py > gpurun_out/refprog.json 2> gpurun_out/refprog.err
timeout -k 10 300 python bench.py --config cfg2 --no-cpu > gpurun_out/bench_cfg2.json 2>/dev/null
