# Round 5 job Y: what taking E off the Viterbi row's B -> E -> J -> B chain could gain at most (VERDICT r04
# item 3): a timing-only build whose B uses the J of one row earlier against HEAD, W = 1 S = 22 on cfg3 /
# cfg4 and the W = 2 S = 19 team on cfg5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_y
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k timeline --timeout 100 --timeout-method thread > $O/timeline_test.txt 2>&1
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --variant vit_w1_s22_ea --rounds 3 abx/tbase/libmsv_hip.so abx/nochain/libmsv_hip.so > $O/ab_cfg3.jsonl

timeout -k 10 300 python tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 2 abx/tbase/libmsv_hip.so abx/nochain/libmsv_hip.so > $O/ab_cfg5.jsonl
