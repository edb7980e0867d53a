# Static first index per lane group: GPU parity, A/B vs ab/blk on cfg2 and cfg3; cfg2 by waves per block.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_first
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/blk/libmsv_hip.so ab/first/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/blk/libmsv_hip.so ab/first/libmsv_hip.so > $O/ab_cfg3.jsonl
for w in 4 8 12 16; do
  timeout -k 10 120 python tools/run_kernel.py --config cfg2 --variant msv_g16_s8_w${w}_p2_d1 --launches 15 --time 20 >> $O/cfg2_waves.jsonl
done
timeout -k 10 200 python tools/wave_timeline.py --config cfg2 > $O/timeline.jsonl
timeout -k 10 200 python tools/wave_timeline.py --config cfg2 --variant msv_g16_s8_w12_p2_d1 >> $O/timeline.jsonl
