#!/bin/bash
# rocprofv3 passes for the MSV kernel on one config (run on the GPU box from the repo root):
#   tools/pmc.sh cfg3 gpurun_out/pmc_cfg3
# One --pmc pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950,
# MI355X_MICROARCH.md "rocprofv3 PMC slots"); kernel-trace/stats in their own pass.
set -e
CFG=${1:-cfg3}
OUT=${2:-gpurun_out/pmc_$CFG}
EXTRA=${3:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
RUN="python3 tools/run_kernel.py --config $CFG --launches 3 $EXTRA"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $RUN
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o run -- $RUN
done
python3 tools/pmc_summary.py "$OUT" "$CFG" > "$OUT/summary.json"
cat "$OUT/summary.json"
