# Round 5 job D: team kernels with phase A pinned ahead of the polls: parity, interleaved timing on the
# cfg3 / cfg5 survivors, and one PMC pass (VALU count, busy, waits) of vit_w2_s11_e and vit_w2_s19_g.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 120 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
timeout -k 10 200 python tools/vit_tune.py --config cfg3 --longest-first --rounds 3 --variants vit_s22_t5a,vit_w2_s11_e,vit_w2_s11_g,vit_w2_s12_e > $O/tune_cfg3.jsonl 2> $O/tune_cfg3.err
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --longest-first --rounds 2 --variants vit_s38_t7gw4,vit_w2_s19_g,vit_w4_s10_g > $O/tune_cfg5.jsonl 2> $O/tune_cfg5.err
for v in vit_w2_s11_e:cfg3 vit_w2_s19_g:cfg5; do
  var=${v%%:*}; cfg=${v##*:}
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$var/pmc1 -o run -- python3 tools/run_vit.py --config $cfg --launches 2 --variant $var > $O/pmc_$var.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $O/pmc_$var/pmc2 -o run -- python3 tools/run_vit.py --config $cfg --launches 2 --variant $var >> $O/pmc_$var.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc_$var/trace -o run -- python3 tools/run_vit.py --config $cfg --launches 2 --variant $var >> $O/pmc_$var.log 2>&1
  python3 tools/pmc_summary.py $O/pmc_$var ${cfg}_viterbi vit_team_kernel > $O/pmc_$var.json
done
