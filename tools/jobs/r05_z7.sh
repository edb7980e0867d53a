# Round 5 job Z7: team-kernel early exit (HEAD) vs the commit before it, interleaved, in place on cfg3 / cfg5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z7
mkdir -p $O
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --in-place --variant vit_w1_s22_ea --rounds 3 abx/tprev/libmsv_hip.so abx/tearly/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg5 --in-place --variant vit_w2_s19_gb --rounds 2 abx/tprev/libmsv_hip.so abx/tearly/libmsv_hip.so > $O/ab_cfg5.jsonl
