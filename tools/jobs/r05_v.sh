# Round 5 job V: per-wave / per-sequence timeline of the S = 22 pick (where cfg3's fixed ~0.25 ms per launch
# goes, profiles/r05_vit_grain_*.jsonl), the Viterbi GPU tests with the stamp hooks, in-place timing.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_v
mkdir -p $O
timeout -k 10 120 python tools/vit_timeline.py --config cfg3 > $O/timeline.jsonl
timeout -k 10 120 python tools/vit_timeline.py --n 3072 --lmin 400 --lmax 400 >> $O/timeline.jsonl
timeout -k 10 120 python tools/vit_timeline.py --n 24576 --lmin 400 --lmax 400 >> $O/timeline.jsonl
timeout -k 10 120 python tools/vit_timeline.py --config cfg5 >> $O/timeline.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --in-place --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea > $O/tune_cfg3_inplace.jsonl
