# Round 4 job C: Viterbi variants timed on the MSV survivors of cfg3 / cfg5 / cfg2 (bitwise-checked across
# the variants), then the Viterbi GPU tests on the new ascending-pass variants.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --rounds 3 > $O/vit_tune_cfg3.jsonl 2> $O/vit_tune_cfg3.err
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --rounds 2 > $O/vit_tune_cfg5.jsonl 2> $O/vit_tune_cfg5.err
timeout -k 10 200 python tools/vit_tune.py --config cfg2 --rounds 3 > $O/vit_tune_cfg2.jsonl 2> $O/vit_tune_cfg2.err
