#!/bin/bash
# Round 6 job L: the W = 1 S = 22 row at four waves per SIMD (16-wave workgroups): every transition in LDS
# (vit_w1_s22_ec4, LA = 3) and LA = 2 (vit_w1_s22_eb4, spills), bitwise first, then cfg3's survivors in place,
# interleaved fresh processes against the pick vit_w1_s22_ea.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k "every_variant or team_variant_stress" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
for r in 1 2 3; do
  for v in vit_w1_s22_ea vit_w1_s22_ec4 vit_w1_s22_eb4; do
    timeout -k 10 200 python tools/vit_tune.py --config cfg3 --in-place --rounds 1 --variants $v >> $O/cfg3.jsonl
  done
done
echo ok
