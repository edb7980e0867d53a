# Round-2 quick check: GPU parity suite, the default bench line, host->device copy rates.
set -e
O=gpurun_out/r02_check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 120 python tools/micro/h2d_bw.py > $O/h2d.jsonl 2> $O/h2d.err
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/micro/h2d_bw.py > $O/h2d_nosdma.jsonl 2> $O/h2d_nosdma.err
