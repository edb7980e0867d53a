# Round 5 job B: the whole GPU suite after the Viterbi launch-slot / argument-check changes (new tests:
# three streams + host call without sync, bad survivor index, calibration at the bench lengths), the
# filter's length x composition record, and the cfg3 bench line (timed scores checked before the clock pass).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1
timeout -k 10 300 python tools/filter_drift.py --out $O/filter_length_composition.jsonl > $O/filter_drift.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
