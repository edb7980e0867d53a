# Round 6: (1) the W = 2 team exchange, minimal torn-safe form of round 5's protocol (wave 0's E record carries
# its last I: {E, st, I, st}; the boundary is {M, st, D, st}; every stamp word checked) -- r6base (HEAD) vs r6x6 on
# cfg5's survivors, 1600 / 1509 / 2207.hmm bands; (2) cfg2's MSV kernel with the per-row event test as a scalar
# countdown -- r6base vs r6x6: kernel A/B (tools/kernel_ab.py) and the one-wave row time (tools/cfg2_floor.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_d
mkdir -p $O
timeout -k 10 200 python -u tools/kernel_ab.py --config cfg2 --rounds 4 abx/r6base/libmsv_hip.so abx/r6x6/libmsv_hip.so > $O/ab_cfg2.jsonl 2> $O/ab_cfg2.err
for L in r6base r6x6; do MSV_LIB_PATH=$PWD/abx/$L/libmsv_hip.so timeout -k 10 60 python -u tools/cfg2_floor.py > $O/floor_$L.json 2>> $O/floor.err; done
timeout -k 10 240 python -u tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 3 --in-place abx/r6base/libmsv_hip.so abx/r6x6/libmsv_hip.so > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1600.hmm --variant vit_w2_s13_ga4 --rounds 3 abx/r6base/libmsv_hip.so abx/r6x6/libmsv_hip.so > $O/ab_1600.jsonl 2> $O/ab_1600.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1509.hmm --variant vit_w2_s12_ga4 --rounds 3 abx/r6base/libmsv_hip.so abx/r6x6/libmsv_hip.so > $O/ab_1509.jsonl 2> $O/ab_1509.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 2207.hmm --variant vit_w2_s18_gb --rounds 3 abx/r6base/libmsv_hip.so abx/r6x6/libmsv_hip.so > $O/ab_2207.jsonl 2> $O/ab_2207.err
