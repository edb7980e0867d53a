# Round 5 job G: PMC of the cfg5 team kernel (vit_w2_s19_g) and the uniform-state A/B of the single-wave kernel.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_g
mkdir -p $O
i=0
for g in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o run -- python3 tools/run_vit.py --config cfg5 --launches 2 >> $O/pmc.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/run_vit.py --config cfg5 --launches 2 >> $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O cfg5_viterbi vit_team_kernel > $O/pmc_cfg5.json
timeout -k 10 400 python tools/vit_ab.py --config cfg3 --variant vit_s22_t5a --rounds 3 abx/base/libmsv_hip.so abx/new/libmsv_hip.so > $O/ab_uniform_cfg3.jsonl
