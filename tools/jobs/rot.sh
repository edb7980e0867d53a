# Rotating residue slots: GPU parity, then A/B against the previous build on the bench configs and on
# the latency plan of 1400.hmm (2048 sequences, G = 64 S = 24).
#   gpurun -- 'bash tools/jobs/rot.sh brs rot'
set -e
O=gpurun_out/rot
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
CONFIGS="cfg2 cfg3 cfg5" REPS=2 bash tools/jobs/ab.sh "$@"
for n in "$@"; do
  MSV_LIB_PATH=$PWD/ab/$n/libmsv_hip.so timeout -k 10 120 python tools/tune.py --profile 1400.hmm --n 2048 --seed 1000 \
    --rounds 3 --reps 5 --variants msv_g64_s24_w16_p6_d1 2>/dev/null | sed "s/^/$n /" | tee -a $O/lat_1400.jsonl
done
