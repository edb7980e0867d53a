# Latency-plan threshold re-check after the residue blocks / static first indices: 1400.hmm main vs
# latency variant at 1k..16k sequences; 2405.hmm and 1901.hmm (no latency plan today) at 3..2k.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_lat
mkdir -p $O
for n in 1024 4096 8192 16384; do
timeout -k 10 200 python tools/tune.py --profile 1400.hmm --n $n --lmin 300 --lmax 500 --seed 2 --rounds 2 --reps 5 --variants msv_g16_s88_w16_p2_d1,msv_g64_s24_w16_p6_d1 > $O/lat_1400_$n.log 2>&1
done
for n in 3 256 2048; do
timeout -k 10 200 python tools/tune.py --profile 1901.hmm --n $n --lmin 300 --lmax 3500 --seed 2 --rounds 2 --reps 3 --variants msv_g32_s60_w16_p2_d1,msv_g64_s32_w16_p2_d1,msv_g64_s34_a32_w16_p2_d1 > $O/lat_1901_$n.log 2>&1
done
