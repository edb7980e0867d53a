set -e
O=gpurun_out/r02_xrow
mkdir -p $O
timeout -k 10 400 python tools/kernel_ab.py --config cfg2 --rounds 4 ab/new/libmsv_hip.so ab/xrow2/libmsv_hip.so > $O/kab_cfg2.jsonl 2> $O/kab_cfg2.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_parity.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
