# Round 5 job C: first GPU run of the team kernels (vit_team.hip): parity (every team variant, stress
# models), then interleaved timing against the single-wave picks on the cfg3 / cfg5 survivors.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 120 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
timeout -k 10 200 python tools/vit_tune.py --config cfg3 --longest-first --rounds 3 --variants vit_s22_t5a,vit_w2_s11_e,vit_w2_s11_g,vit_w2_s12_e,vit_w3_s13_g,vit_w4_s10_g > $O/tune_cfg3.jsonl 2> $O/tune_cfg3.err
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --longest-first --rounds 2 --variants vit_s38_t7gw4,vit_w2_s19_g,vit_w3_s13_g,vit_w4_s10_g > $O/tune_cfg5.jsonl 2> $O/tune_cfg5.err
