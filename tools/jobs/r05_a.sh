# Round 5 job A: PMC attribution of the Viterbi stage's S = 38 kernel on the cfg5 survivors
# (vit_kernel<38,7,false,false,4,3,false>, tools/run_vit.py) -- the counters the round-5 rewrite aims at --
# and the Viterbi GPU tests at HEAD.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.log 2>&1
RUN="python3 tools/run_vit.py --config cfg5 --launches 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $RUN > $O/trace.log 2>&1
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- $RUN > $O/pmc$i.log 2>&1
done
python3 tools/pmc_summary.py $O cfg5_viterbi vit_kernel > $O/summary.json
cat $O/summary.json
