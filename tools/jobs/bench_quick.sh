set -e
timeout -k 10 300 python bench.py --config ${1:-cfg2} ${2:-} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
