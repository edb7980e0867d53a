# Round 6 closing job, part B (at the final HEAD): rocprofv3 kernel-trace summaries + exact-variant windows of
# the cfg3 / cfg5 bench commands, HBM + instruction counters of the cfg3 MSV kernel (tools/pmc.sh), PMC of the
# two Viterbi picks on their survivors (cfg3 vit_w1_s22_ea, cfg5 vit_w2_s19_gb).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_final_b
mkdir -p $O
for c in cfg3 cfg5; do
  case $c in cfg5) ST=10;; *) ST=20;; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python3 bench.py --config $c --no-cpu --no-clock --steps $ST > $O/bench_${c}_rocprof.json 2> $O/bench_${c}_rocprof.err
  V=$(python3 -c "import json;print(json.load(open('$O/bench_${c}_rocprof.json'))['config']['kernel_variant'])")
  python3 tools/rocprof_window.py $(find $O/trace_$c -name '*kernel_trace.csv') --variant $V --last $ST > $O/window_$c.json
  cp $(find $O/trace_$c -name '*kernel_stats.csv') $O/kernel_stats_$c.csv
  rm -rf $O/trace_$c
done
bash tools/pmc.sh cfg3 $O/pmc_cfg3 > $O/pmc_cfg3.log 2>&1
cp $O/pmc_cfg3/summary.json $O/pmc_cfg3.json
rm -rf $O/pmc_cfg3
for c in cfg3 cfg5; do
  P=$O/vpmc_$c
  mkdir -p $P
  i=0
  for g in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 150 rocprofv3 --pmc $g --output-format csv -d $P/pmc$i -o run -- python3 tools/run_vit.py --config $c --launches 3 >> $P/pmc.log 2>&1
  done
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 tools/run_vit.py --config $c --launches 3 >> $P/pmc.log 2>&1
  python3 tools/pmc_summary.py $P ${c}_viterbi vit_team_kernel > $O/pmc_vit_$c.json
  rm -rf $P/pmc1 $P/pmc2 $P/pmc3 $P/trace
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q -k "many_blocks or clamped or filter_select" --timeout 150 --timeout-method thread > $O/pytest_new.log 2>&1
