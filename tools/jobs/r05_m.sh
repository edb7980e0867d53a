# Round 5 job M: phase-A transitions as paired float4 LDS reads (one ds_read_b128 per pair and chunk) -- A/B
# of the team picks against the previous layout (vit_ab.py: fresh process per build, interleaved), parity.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
timeout -k 10 500 python tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 3 abx/tbase/libmsv_hip.so abx/tnew/libmsv_hip.so > $O/ab_pairs_cfg5.jsonl
