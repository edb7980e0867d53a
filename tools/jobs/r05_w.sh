# Round 5 job W: the team kernel's next-sequence atomic taken after the first row (VIT_TAKE_LATE) and the
# youngest-wave cutoff (VIT_YOUNG_CUT = 2, 4: quarters of the team count) -- interleaved A/B on cfg3 (S = 22,
# W = 1) and cfg5 (W = 2), the cfg3 timelines, the Viterbi GPU tests on the cutoff build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_w
mkdir -p $O
timeout -k 10 400 python tools/vit_ab.py --config cfg3 --variant vit_w1_s22_ea --rounds 3 abx/tbase/libmsv_hip.so abx/tlate/libmsv_hip.so abx/ty2/libmsv_hip.so abx/ty4/libmsv_hip.so > $O/ab_cfg3.jsonl
for b in tlate ty2 ty4; do
  MSV_LIB_PATH=$PWD/abx/$b/libmsv_hip.so timeout -k 10 120 python tools/vit_timeline.py --config cfg3 > $O/timeline_$b.jsonl
done
timeout -k 10 400 python tools/vit_ab.py --config cfg5 --variant vit_w2_s19_gb --rounds 2 abx/tbase/libmsv_hip.so abx/tlate/libmsv_hip.so > $O/ab_cfg5.jsonl
MSV_LIB_PATH=$PWD/abx/ty2/libmsv_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests_ty2.txt 2>&1
