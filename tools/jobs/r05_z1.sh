# Round 5 job Z1: the team kernels' unconditional first lazy-F pass (kTeamEarlyD slots, 8 at HEAD) against
# 0 (ballot first), 4 and 12 -- W = 1 S = 22 on cfg3, W = 2 S = 19 on cfg5; bitwise by construction (the
# lazy-F passes only raise lower bounds to the serial chain), checked by the Viterbi tests on ed0.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z1
mkdir -p $O
MSV_LIB_PATH=$PWD/abx/ed0/libmsv_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k "team or every_profile or long_delete" --timeout 200 --timeout-method thread > $O/vit_tests_ed0.txt 2>&1
timeout -k 10 400 python tools/vit_ab.py --config cfg3 --variant vit_w1_s22_ea --rounds 3 abx/tbase/libmsv_hip.so abx/ed0/libmsv_hip.so abx/ed4/libmsv_hip.so abx/ed12/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 400 python tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 2 abx/tbase/libmsv_hip.so abx/ed0/libmsv_hip.so abx/ed4/libmsv_hip.so abx/ed12/libmsv_hip.so > $O/ab_cfg5.jsonl
