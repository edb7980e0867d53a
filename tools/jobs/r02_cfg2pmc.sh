# cfg2 latency counters: L1->L2 read latency, L2 hit rate, per-row wait attribution.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_cfg2pmc
mkdir -p $O
RUN="python3 tools/run_kernel.py --config cfg2 --launches 5"
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
i=0
for grp in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc$i" -o run -- $RUN > $O/pmc$i.log 2>&1 || echo "pass $i failed" >> $O/failed.txt
done
