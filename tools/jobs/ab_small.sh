# A/B of library builds on the short-row paths: cfg2 (100.hmm x 10k, G=16 S=8) through bench.py and the
# latency plan of 1400.hmm (2048 sequences, G=64 S=24) through tools/tune.py.
#   gpurun -- 'bash tools/jobs/ab_small.sh base new'
set -e
O=gpurun_out/ab_small
mkdir -p $O
CONFIGS="cfg2" REPS=3 bash tools/jobs/ab.sh "$@"
for r in 1 2; do
  for n in "$@"; do
    MSV_LIB_PATH=$PWD/ab/$n/libmsv_hip.so timeout -k 10 120 python tools/tune.py --profile 1400.hmm --n 2048 --seed 1000 \
      --rounds 3 --reps 5 --variants msv_g64_s24_w16_p6_d1 2>/dev/null | grep '"order": true' | sed "s/^/$n /" | tee -a $O/lat_1400.jsonl
  done
done
