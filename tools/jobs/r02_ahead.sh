# Next-index fetch a few rows before the end (vs half-way): interleaved kernel A/B on cfg3 and cfg5,
# lookahead 8+256/S (ahead), 24+768/S (ahead3), 4+128/S (aheadh) against half-way (ab/host).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_ahead
mkdir -p $O
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/host/libmsv_hip.so ab/ahead/libmsv_hip.so ab/ahead3/libmsv_hip.so ab/aheadh/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 400 python tools/kernel_ab.py --config cfg5 --rounds 2 --warm 5 --time 5 ab/host/libmsv_hip.so ab/ahead/libmsv_hip.so ab/ahead3/libmsv_hip.so > $O/ab_cfg5.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 400.hmm --rounds 2 ab/host/libmsv_hip.so ab/ahead/libmsv_hip.so ab/ahead3/libmsv_hip.so > $O/ab_400.jsonl
