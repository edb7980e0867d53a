# Round 5 job ZD: two rows per loop trip for the LA team variants (the picks from 1,601 to 2,432 states) vs
# one row: 7,000 random sequences on 1600 / 1705 / 1901 / 2138 / 2207.hmm, cfg5's survivors in place; the
# Viterbi tests on the new in-tree build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
for pv in 1600.hmm:vit_w2_s13_ga 1705.hmm:vit_w2_s14_ga 1901.hmm:vit_w2_s15_ga 2138.hmm:vit_w2_s17_gb 2207.hmm:vit_w2_s18_gb; do
  p=${pv%%:*}; v=${pv##*:}
  timeout -k 10 200 python tools/vit_ab.py --n 7000 --profile $p --variant $v --rounds 2 abx/one/libmsv_hip.so abx/two/libmsv_hip.so >> $O/ab_bands.jsonl
done
timeout -k 10 300 python tools/vit_ab.py --config cfg5 --in-place --variant vit_w2_s19_gb --rounds 2 abx/one/libmsv_hip.so abx/two/libmsv_hip.so > $O/ab_cfg5.jsonl
