# Round 6: the lone-sequence row time of the W = 1 pick vs a W = 2 team (vit_w2_s11_g) on 1400.hmm -- batches
# small enough that every wave / team has its SIMD(s) to itself (512 x 400 rows), and for reference 3,072 and
# 7,261 sequences: what a W = 2 tail phase could gain.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_j
mkdir -p $O
for N in 256 512 1536 3072; do
  timeout -k 10 120 python -u tools/vit_tune.py --profile 1400.hmm --n $N --lmin 400 --lmax 400 --rounds 3 --reps 5 --variants vit_w1_s22_ea,vit_w2_s11_g,vit_s22_t5a >> $O/lone_rows.jsonl 2>> $O/lone_rows.err
done
