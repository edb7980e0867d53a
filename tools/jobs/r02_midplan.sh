# Mid plan (G = 32) for mid-size batches: parity tests, then the automatic plan over all profiles at 9k/12k/16k sequences.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_midplan
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -k "mid_plan or every_plan or every_variant or latency_plan" > $O/pytest.log 2>&1
for n in 9000 12000 16000; do
timeout -k 10 300 python tools/profile_sweep.py --config cfg3 --n $n --time 20 >> $O/sweep.jsonl
done
