# Round 5 job Q: the S = 22 pick vs vit_s22_t5a in bench.py's setting (whole cfg3 / cfg4 batch in place,
# survivors from msv_filter_select_device) and in the compacted setting, one box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_q
mkdir -p $O
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --in-place --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea,vit_w1_s22_eb > $O/tune_cfg3_inplace.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --longest-first --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea,vit_w1_s22_eb > $O/tune_cfg3.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --in-place --rounds 2 --variants vit_s38_t7gw4,vit_w2_s19_gb > $O/tune_cfg5_inplace.jsonl
