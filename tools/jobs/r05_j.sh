# Round 5 job J: the team kernel at W = 1 (one wave per sequence, phase-A/DM transitions and match scores in
# LDS, three waves per SIMD) against vit_kernel.hip's S = 20/22 picks: parity, cfg3 survivors, 1200.hmm band.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_viterbi.py -x -q --timeout 200 --timeout-method thread -k "team or (every_variant and vit_w)" > $O/team_tests.txt 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --longest-first --rounds 3 --variants vit_s22_t5a,vit_w1_s22_eb,vit_w1_s22_ea,vit_w1_s22_gb,vit_w2_s11_ea4 > $O/tune_cfg3.jsonl
timeout -k 10 150 python tools/vit_tune.py --n 7000 --lmin 300 --lmax 500 --rounds 2 --profile 1200.hmm --variants vit_s20_t5a,vit_w1_s20_eb > $O/tune_bands.jsonl
