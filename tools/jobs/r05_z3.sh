# Round 5 job Z3: the Viterbi launches' first sequences dealt one per workgroup (item = w * grid + block) and
# at least one workgroup per CU, vs HEAD (a workgroup's waves took consecutive items, and a host list of n
# sequences got ceil(n / waves) workgroups): cfg2's 260 survivors (latency-bound) compacted and in place, and
# the throughput picks on cfg3 / cfg5 for regressions; the Viterbi GPU tests on the new build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --variant vit_s2_t7 --rounds 3 abx/tbase/libmsv_hip.so abx/spread/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s2_t7 --rounds 3 abx/tbase/libmsv_hip.so abx/spread/libmsv_hip.so > $O/ab_cfg2_inplace.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s4_t7 --rounds 2 abx/tbase/libmsv_hip.so abx/spread/libmsv_hip.so > $O/ab_cfg2_inplace_s4.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --in-place --variant vit_w1_s22_ea --rounds 3 abx/tbase/libmsv_hip.so abx/spread/libmsv_hip.so > $O/ab_cfg3.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg5 --in-place --variant vit_w2_s19_gb --rounds 2 abx/tbase/libmsv_hip.so abx/spread/libmsv_hip.so > $O/ab_cfg5.jsonl
