# Round 5 job N: W = 1 team forms of the S = 22 row (paired LDS transitions) against vit_s22_t5a, cfg3 survivors.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread -k "team and w1" > $O/team_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --longest-first --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea,vit_w1_s22_eb,vit_w1_s22_e,vit_w1_s22_ea2 > $O/tune_cfg3.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg4 --longest-first --rounds 2 --variants vit_s22_t5a,vit_w1_s22_ea,vit_w1_s22_eb > $O/tune_cfg4.jsonl
# DM_IN chunk pairs as float4 LDS reads (LA = 2 variants), A/B against HEAD (paired phase A only)
timeout -k 10 500 python tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 3 abx/tbase/libmsv_hip.so abx/tnew/libmsv_hip.so > $O/ab_dmpairs_cfg5.jsonl
