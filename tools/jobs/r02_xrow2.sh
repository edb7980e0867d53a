# Whole-row-ring throughput plans: GPU suite, automatic plans at 10k / 30k / 100k over all profiles.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_xrow2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for n in 10000 30000 100000; do
timeout -k 10 300 python tools/profile_sweep.py --config cfg3 --n $n --time 20 >> $O/sweep.jsonl
done
