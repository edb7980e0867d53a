# Round 5 job I: four-waves-per-SIMD team variants (S = 11, 12) and three-wave S = 13/14 ones against the
# single-wave picks (cfg3 survivors; 1509/1600/1705.hmm bands), and a PMC pass of the cfg5 pick vit_w2_s19_gb.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --longest-first --rounds 3 --variants vit_s22_t5a,vit_w2_s11_ea4,vit_w2_s11_ga4,vit_w2_s11_ea,vit_w2_s11_e > $O/tune_cfg3.jsonl
T="timeout -k 10 150 python tools/vit_tune.py --n 7000 --lmin 300 --lmax 500 --rounds 2"
$T --profile 1509.hmm --variants vit_w2_s12_g,vit_w2_s12_ga4 > $O/tune_bands.jsonl
$T --profile 1600.hmm --variants vit_s26_t0g,vit_w2_s13_ga >> $O/tune_bands.jsonl
$T --profile 1705.hmm --variants vit_s28_t0g,vit_w2_s14_ga >> $O/tune_bands.jsonl
i=0
for g in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d $O/pmc$i -o run -- python3 tools/run_vit.py --config cfg5 --launches 2 >> $O/pmc.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/run_vit.py --config cfg5 --launches 2 >> $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O cfg5_viterbi vit_team_kernel > $O/pmc_cfg5.json
