# Round 5 job P: PMC of the new S = 22 pick (vit_w1_s22_ea) on the cfg3 survivors; the whole Viterbi GPU file;
# bench cfg3 and cfg4 lines (their viterbi_stage now runs the W = 1 team kernel).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
i=0
for g in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o run -- python3 tools/run_vit.py --config cfg3 --launches 3 >> $O/pmc.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/run_vit.py --config cfg3 --launches 3 >> $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O cfg3_viterbi vit_team_kernel > $O/pmc_cfg3.json
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 250 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
