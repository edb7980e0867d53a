set -e
for n in 512 2048 4096 8192; do
timeout -k 10 200 python tools/tune.py --profile 1400.hmm --n $n --lmin 300 --lmax 500 --seed 2 --rounds 2 --reps 5 --variants msv_g16_s88_w16_p2_d1,msv_g64_s24_w16_p6_d1 > gpurun_out/lat_1400_$n.log 2>&1
timeout -k 10 200 python tools/tune.py --profile 100.hmm --n $n --lmin 300 --lmax 500 --seed 1 --rounds 2 --reps 5 --variants msv_g16_s8_w4_p2_d1,msv_g64_s4_w16_p1_d1,msv_g64_s8_w16_p2_d1 > gpurun_out/lat_100_$n.log 2>&1
done
timeout -k 10 200 python tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1 --rounds 2 --reps 5 --variants msv_g16_s8_w4_p2_d1,msv_g64_s4_w16_p1_d1,msv_g64_s8_w16_p2_d1 > gpurun_out/lat_100_10000.log 2>&1
