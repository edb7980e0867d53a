# Round 5 job Z8: the team-kernel early exit where it applies -- a device-count launch of few survivors
# (cfg3's first 10,000 sequences: ~730 survivors for 3,072 waves) -- vs the commit before it, in place.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z8
mkdir -p $O
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --config-n 10000 --in-place --variant vit_w1_s22_ea --rounds 3 abx/tprev/libmsv_hip.so abx/tearly/libmsv_hip.so > $O/ab_cfg3_10k.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg5 --config-n 5000 --in-place --variant vit_w2_s19_gb --rounds 3 abx/tprev/libmsv_hip.so abx/tearly/libmsv_hip.so > $O/ab_cfg5_5k.jsonl
