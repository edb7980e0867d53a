# Round 6: wave 1 of a W = 2 team reads wave 0's E record right after the boundary poll, under its lazy-F pass,
# instead of polling it after: r6x11 = round 5's protocol + that; r6x10 = the same on the {E,st,I,st}/{M,st,D,st}
# records; vs r6base (HEAD), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_f
mkdir -p $O
L="abx/r6base/libmsv_hip.so abx/r6x11/libmsv_hip.so abx/r6x10/libmsv_hip.so"
timeout -k 10 300 python -u tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 3 --in-place $L > $O/ab_cfg5.jsonl 2> $O/ab_cfg5.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 2207.hmm --variant vit_w2_s18_gb --rounds 2 $L > $O/ab_2207.jsonl 2> $O/ab_2207.err
timeout -k 10 200 python -u tools/vit_ab.py --n 7000 --profile 1600.hmm --variant vit_w2_s13_ga4 --rounds 2 $L > $O/ab_1600.jsonl 2> $O/ab_1600.err
