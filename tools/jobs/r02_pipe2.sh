set -e
O=gpurun_out/r02_pipe2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 500 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/base/libmsv_hip.so ab/new/libmsv_hip.so > $O/kab_cfg3.jsonl 2> $O/kab_cfg3.err
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 2 ab/base/libmsv_hip.so ab/new/libmsv_hip.so > $O/kab_cfg2.jsonl 2> $O/kab_cfg2.err
timeout -k 10 300 python tools/host_pipeline_sweep.py --config cfg3 > $O/sweep_cfg3.jsonl 2> $O/sweep_cfg3.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
