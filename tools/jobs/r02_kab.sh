# Kernel-only A/B of two library builds (ab/base, ab/new), interleaved processes.
set -e
O=gpurun_out/r02_kab
mkdir -p $O
timeout -k 10 500 python tools/kernel_ab.py --config cfg3 --rounds 4 ab/base/libmsv_hip.so ab/new/libmsv_hip.so > $O/kab_cfg3.jsonl 2> $O/kab_cfg3.err
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 2 ab/base/libmsv_hip.so ab/new/libmsv_hip.so > $O/kab_cfg2.jsonl 2> $O/kab_cfg2.err
