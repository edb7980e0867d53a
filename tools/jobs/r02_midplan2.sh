# Mid plan extended to S >= 40: GPU suite, then the automatic plans over all profiles at 3k..16k sequences.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_midplan2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for n in 3000 6000 9000 12000 16000; do
timeout -k 10 300 python tools/profile_sweep.py --config cfg3 --n $n --time 20 >> $O/sweep.jsonl
done
