# Small profiles at large batch sizes: is the one dequeue counter the bound?  GPU P-value calibration test.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_rate
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "calibration" --timeout 240 --timeout-method thread > $O/pytest_calib.log 2>&1
for n in 10000 100000 1000000; do
timeout -k 10 200 python tools/run_kernel.py --config cfg2 --n $n --launches 5 --time 10 >> $O/rate.jsonl
done
timeout -k 10 200 python tools/run_kernel.py --config cfg2 --profile 400.hmm --n 1000000 --launches 3 --time 5 >> $O/rate.jsonl
timeout -k 10 200 python tools/run_kernel.py --config cfg2 --profile 400.hmm --n 100000 --launches 3 --time 5 >> $O/rate.jsonl
