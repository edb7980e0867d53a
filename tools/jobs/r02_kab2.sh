set -e
O=gpurun_out/r02_kab2
mkdir -p $O
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/new/libmsv_hip.so ab/noev/libmsv_hip.so > $O/kab_cfg2.jsonl 2> $O/kab_cfg2.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
