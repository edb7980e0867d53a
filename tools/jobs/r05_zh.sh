# Round 5 job ZH: W = 1 team rows two per trip (VIT_TEAM_TWO_ROWS_W1 build: no spills for w1_s22_eb, s20_eb,
# s12..s18_ea) against the picks (in-tree build), alternating fresh processes: cfg3 in place (w1_s22_ea pick vs
# w1_s22_eb two rows), 1200.hmm (s20_t5a vs w1_s20_eb), 1001.hmm (s16_t7 vs w1_s16_ea), 700.hmm (s12_t7 vs
# w1_s12_ea), 7,000 random sequences.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_zh
mkdir -p $O
L2=$PWD/abx/w1two/libmsv_hip.so
for r in 1 2 3; do
  timeout -k 10 200 python tools/vit_tune.py --config cfg3 --in-place --rounds 1 --variants vit_w1_s22_ea >> $O/cfg3_head.jsonl
  MSV_LIB_PATH=$L2 timeout -k 10 200 python tools/vit_tune.py --config cfg3 --in-place --rounds 1 --variants vit_w1_s22_eb >> $O/cfg3_w1two.jsonl
done
for pv in 1200.hmm:vit_s20_t5a:vit_w1_s20_eb 1001.hmm:vit_s16_t7:vit_w1_s16_ea 700.hmm:vit_s12_t7:vit_w1_s12_ea; do
  IFS=: read p a b <<< "$pv"
  for r in 1 2; do
    timeout -k 10 200 python tools/vit_tune.py --profile $p --n 7000 --rounds 1 --variants $a >> $O/bands_head.jsonl
    MSV_LIB_PATH=$L2 timeout -k 10 200 python tools/vit_tune.py --profile $p --n 7000 --rounds 1 --variants $b >> $O/bands_w1two.jsonl
  done
done
