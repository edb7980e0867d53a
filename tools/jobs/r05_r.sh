# Round 5 job R: is the in-place gap the survivors' order?  bench.py's setting with the device survivors list
# as msv_filter_select_device makes it (stretches of the MSV order, appended in atomic order) vs re-listed
# exactly longest first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_r
mkdir -p $O
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --in-place --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea > $O/tune_cfg3_inplace.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --in-place --sort-select --rounds 3 --variants vit_s22_t5a,vit_w1_s22_ea > $O/tune_cfg3_inplace_sorted.jsonl
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --in-place --sort-select --rounds 2 --variants vit_w2_s19_gb > $O/tune_cfg5_inplace_sorted.jsonl
