# Round 5 job F: team kernels with wave-uniform sequence/stamp state (scalar branches and polls), now the
# picks for 1409-1536, 1793-1920 and 2049-2432 states: the Viterbi GPU tests, cfg5 / band timing, PMC.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --longest-first --rounds 2 --variants vit_s38_t7gw4,vit_w2_s19_g > $O/tune_cfg5.jsonl
timeout -k 10 200 python tools/vit_tune.py --config cfg3 --longest-first --rounds 2 --variants vit_s22_t5a,vit_w2_s11_e,vit_w2_s12_g > $O/tune_cfg3.jsonl
T="timeout -k 10 150 python tools/vit_tune.py --n 7000 --lmin 300 --lmax 500 --rounds 2"
$T --profile 1509.hmm --variants vit_s24_t0g,vit_w2_s12_g > $O/tune_bands.jsonl
$T --profile 1901.hmm --variants vit_s30_t0g,vit_w2_s15_g >> $O/tune_bands.jsonl
$T --profile 2138.hmm --variants vit_s34_t7gw4,vit_w2_s17_g >> $O/tune_bands.jsonl
for g in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU"; do
  timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d $O/pmc/p$(echo $g | cut -c1-12 | tr ' ' _) -o run -- python3 tools/run_vit.py --config cfg5 --launches 2 >> $O/pmc.log 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc/trace -o run -- python3 tools/run_vit.py --config cfg5 --launches 2 >> $O/pmc.log 2>&1
python3 tools/pmc_summary.py $O/pmc cfg5_viterbi vit_team_kernel > $O/pmc_cfg5.json
# the single-wave kernels with wave-uniform sequence state (readfirstlane), A/B against the committed build
timeout -k 10 400 python tools/vit_ab.py --config cfg3 --variant vit_s22_t5a --rounds 3 abx/base/libmsv_hip.so abx/new/libmsv_hip.so > $O/ab_uniform_cfg3.jsonl
