set -e
O=gpurun_out/r02_tune2
mkdir -p $O
timeout -k 10 400 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1000 --rounds 3 --reps 5 \
  --variants msv_g16_s8_w4_p2_d1,msv_g32_s4_w8_p1_d1,msv_g32_s4_w16_p1_d1,msv_g32_s8_w8_p2_d1,msv_g64_s4_w16_p1_d1,msv_g16_s8_w8_p2_d1 > $O/tune_cfg2.jsonl 2> $O/tune_cfg2.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "every_variant or latency_plan or homolog" --timeout 240 --timeout-method thread > $O/pytest_variants.log 2>&1
