# Per-wave timeline of cfg2 (100.hmm x 10k) and of 1400.hmm x 2048 (latency plan): ns per row, waves per SIMD.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_tl2
mkdir -p $O
timeout -k 10 200 python tools/wave_timeline.py --config cfg2 > $O/timeline.jsonl
timeout -k 10 200 python tools/wave_timeline.py --config cfg2 --variant msv_g16_s8_w16_p2_d1 >> $O/timeline.jsonl
timeout -k 10 200 python tools/wave_timeline.py --config cfg3 --n 2048 >> $O/timeline.jsonl
timeout -k 10 200 python tools/wave_timeline.py --config cfg3 --n 100 >> $O/timeline.jsonl
