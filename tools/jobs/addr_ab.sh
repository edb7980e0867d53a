# GPU parity, then the one-VALU row addresses (ab/new: v_mad_u32_u24 for the LDS row and the split B
# table) against the previous build (ab/base) on cfg3 / cfg5 / cfg2, interleaved.
set -e
O=gpurun_out/addr_ab
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
CONFIGS="cfg3 cfg5 cfg2" REPS=3 STEPS=20 bash tools/jobs/ab.sh base new
