#!/bin/bash
# Round 6 job N: one wave per sequence for 2405.hmm (S = 38, W = 1): every transition in LDS (LA = 3), match
# scores from L2, two waves per SIMD (vit_w1_s38_gc2, 226 VGPRs, no scratch), against cfg5's pick vit_w2_s19_gb;
# bitwise first, then cfg5's survivors in place, interleaved fresh processes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k "every_variant or team_variant_stress" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
for r in 1 2 3; do
  for v in vit_w2_s19_gb vit_w1_s38_gc2; do
    timeout -k 10 250 python tools/vit_tune.py --config cfg5 --in-place --rounds 1 --variants $v >> $O/cfg5.jsonl
  done
done
echo ok
