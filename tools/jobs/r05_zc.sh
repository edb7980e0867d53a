# Round 5 job ZC: two rows per loop trip for the two-wave teams (no spills at S = 19; the one-row loop copies
# values at its back edge) vs HEAD, in place on cfg5; the team stress tests on the A/B build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zc
mkdir -p $O
MSV_LIB_PATH=$PWD/abx/tworows/libmsv_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k "team or every_variant or three_streams" --timeout 200 --timeout-method thread > $O/vit_tests_tworows.txt 2>&1
timeout -k 10 400 python tools/vit_ab.py --config cfg5 --in-place --variant vit_w2_s19_gb --rounds 3 abx/base/libmsv_hip.so abx/tworows/libmsv_hip.so > $O/ab_cfg5.jsonl
