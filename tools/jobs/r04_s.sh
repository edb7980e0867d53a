# Round 4 job S: PMC attribution (final build) of the Viterbi stage's kernel on the cfg3 survivors (tools/run_vit.py):
# one kernel-trace pass, then one --pmc pass per counter group (SQ only, <= 4 per pass).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_s
mkdir -p $O
RUN="python3 tools/run_vit.py --config cfg3 --launches 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $RUN > $O/trace.log 2>&1
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- $RUN > $O/pmc$i.log 2>&1
done
python3 tools/pmc_summary.py $O cfg3_viterbi vit_kernel > $O/summary.json
