# Round 5 job X: can a second, concurrent launch fill the Viterbi launch's drain tail?  cfg3's survivors split
# into a head (the S = 22 pick) and a tail of K sequences (small-workgroup two-wave teams) on a second stream.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -x -q -k "every_variant or team" --timeout 200 --timeout-method thread > $O/vit_tests.txt 2>&1
timeout -k 10 200 python tools/vit_concurrent.py --config cfg3 --tail vit_w2_s11_g1 > $O/conc_g1.jsonl
timeout -k 10 200 python tools/vit_concurrent.py --config cfg3 --tail vit_w2_s11_g2 > $O/conc_g2.jsonl
timeout -k 10 200 python tools/vit_concurrent.py --config cfg3 --tail vit_w2_s11_g --ks 0,512,1024,2048 > $O/conc_g6.jsonl
