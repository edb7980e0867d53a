# Round 4 job L: Viterbi prefetch-depth / pass-order candidates at S = 22 and S = 38 (parity first).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread -k "every_variant or long_delete or reduction" > $O/pytest_vit.log 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --longest-first --rounds 4 --variants vit_s22_t5a,vit_s22_t5,vit_s22_t5a2,vit_s22_t5p2 > $O/tune_cfg3.jsonl 2> $O/tune.err
timeout -k 10 400 python tools/vit_tune.py --config cfg5 --longest-first --rounds 2 --reps 3 --variants vit_s38_t7gw4,vit_s38_t7gw4p2,vit_s38_t7gw4p4,vit_s38_t7gw4a,vit_s38_t0g4 > $O/tune_cfg5.jsonl 2>> $O/tune.err
