# Round 5 job Z6: team-kernel workgroups without a sequence leave at once (as the single-wave kernel's):
# Viterbi GPU tests, in-place timing of the picks on cfg3 / cfg5, bench cfg5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --in-place --rounds 3 --variants vit_w1_s22_ea > $O/tune_cfg3.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --in-place --rounds 2 --variants vit_w2_s19_gb > $O/tune_cfg5.jsonl
timeout -k 10 200 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
