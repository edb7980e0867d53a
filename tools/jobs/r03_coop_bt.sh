# Cooperative plan with Bt computed one region ahead: GPU suite, single-sequence sweep, reference programs.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_coop_bt
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python tools/coop_sweep.py --profile 1400.hmm --ns 1,3,64,256 --lmin 3500 --lmax 3500 > $O/sweep.jsonl 2> $O/sweep.err
timeout -k 10 200 python tools/coop_sweep.py --profile 2405.hmm --ns 1,3,64 --lmin 3500 --lmax 3500 >> $O/sweep.jsonl 2>> $O/sweep.err
timeout -k 10 300 python tools/bench_reference_programs.py > $O/reference_programs.json 2> $O/reference_programs.err
