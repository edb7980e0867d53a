# GPU parity, then the lane-contiguous split B table (ab/new) against the previous build (ab/base) on cfg5.
set -e
O=gpurun_out/splitb_ab
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
CONFIGS="cfg5" REPS=3 STEPS=10 bash tools/jobs/ab.sh base new
