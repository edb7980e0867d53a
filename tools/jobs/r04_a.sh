# Round 4 job A: the Viterbi stage's GPU tests, the clock-stamp A/B (cfg3, cfg2), cfg2's floor and D=2 /
# 8x16 A/B.  Each step under its own time limit; the first failure ends the job.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
timeout -k 10 240 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/base/libmsv_hip.so ab/stamp/libmsv_hip.so > $O/ab_stamp_cfg3.jsonl 2> $O/ab_stamp.err
timeout -k 10 150 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/stamp/libmsv_hip.so > $O/ab_stamp_cfg2.jsonl 2>> $O/ab_stamp.err
timeout -k 10 200 python tools/cfg2_floor.py --out $O/cfg2_floor.json > $O/cfg2_floor.log 2>&1
timeout -k 10 300 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1000 --rounds 4 \
  --variants msv_g16_s8_w4_p2_d1,msv_g16_s8_w4_p2_d2,msv_g16_s8_w8_p2_d2,msv_g8_s16_w16_p4_d1,msv_g8_s16_w8_p4_d1,msv_g16_s8_w8_p2_d1 \
  > $O/tune_cfg2.jsonl 2> $O/tune_cfg2.err
