# Round 5 job ZI: the single-wave row lambdas forced inline (a second row-loop instantiation had put the
# M / I / D arrays of S = 14..24 in scratch: 1001.hmm 41 ms, 1200.hmm 34 ms); scratch_bytes per variant test;
# the band timings back; the Viterbi and C-ABI GPU tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zi
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py tests/test_capi.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
for pv in 700.hmm:vit_s12_t7 800.hmm:vit_s14_t7 1001.hmm:vit_s16_t7 1100.hmm:vit_s18_t7 1200.hmm:vit_s20_t5a; do
  p=${pv%%:*}; v=${pv##*:}
  timeout -k 10 200 python tools/vit_tune.py --profile $p --n 7000 --rounds 2 --variants $v >> $O/bands.jsonl
done
