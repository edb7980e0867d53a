# GPU parity + split-layout A/B (2405.hmm, cfg5 shape) + speculative-B timing experiment (cfg2/cfg3 shapes).
#   gpurun -- 'bash tools/jobs/split32.sh'
set -e
O=gpurun_out/split32
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 240 python tools/tune.py --profile 2405.hmm --n 100000 --lmin 1500 --lmax 2500 --seed 4000 --rounds 2 --reps 2 \
  --variants msv_g32_s76_a64_w16_p2_d1,msv_g32_s76_a64_w12_p2_d1,msv_g64_s38_a32_w16_p2_d1,msv_g64_s40_w16_p2_d1 \
  > $O/tune_2405.jsonl 2> $O/tune_2405.err
cat $O/tune_2405.jsonl
MSV_LIB_PATH=$PWD/ab/exp/libmsv_hip.so timeout -k 10 120 python tools/tune.py --profile 100.hmm --n 10000 --seed 1000 \
  --rounds 3 --reps 5 --variants msv_g16_s8_w4_p2_d1,exp4096_g16_s8_w4_p2_d1 > $O/tune_spec_100.jsonl 2> $O/tune_spec_100.err
cat $O/tune_spec_100.jsonl
MSV_LIB_PATH=$PWD/ab/exp/libmsv_hip.so timeout -k 10 120 python tools/tune.py --profile 1400.hmm --n 100000 --seed 2000 \
  --rounds 3 --reps 3 --variants msv_g16_s88_w16_p2_d1,exp4096_g16_s88_w16_p2_d1 > $O/tune_spec_1400.jsonl 2> $O/tune_spec_1400.err
cat $O/tune_spec_1400.jsonl
timeout -k 10 240 python bench.py --config cfg5 --no-cpu --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
cat $O/bench_cfg5.json
