# Round 5 job ZE: two rows per loop trip for the W = 1 team picks too (S = 22 then spills 20 VGPRs, 8 at one
# row) vs HEAD, in place on cfg3, and 1301.hmm x 7,000.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_ze
mkdir -p $O
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --in-place --variant vit_w1_s22_ea --rounds 3 abx/base/libmsv_hip.so abx/w1two/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 200 python tools/vit_ab.py --n 7000 --profile 1301.hmm --variant vit_w1_s22_ea --rounds 2 abx/base/libmsv_hip.so abx/w1two/libmsv_hip.so > $O/ab_1301.jsonl
