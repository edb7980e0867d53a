# Round 5 job T: where the S = 22 pick loses against cfg4: sequences per wave.  vit_w1_s22_ea on random
# 1400.hmm batches, longest first, at equal lengths (400: no length imbalance, only the last round's
# granularity) and at cfg3's U[300, 500], for 1 .. 24 sequences per wave (3,072 waves); the cfg3 bench line
# (viterbi_stage now the median of its launches, every launch listed).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_t
mkdir -p $O
for n in 3072 6144 7261 9216 12288 24576 73728; do
  timeout -k 10 120 python tools/vit_tune.py --profile 1400.hmm --n $n --lmin 400 --lmax 400 --longest-first --rounds 2 --variants vit_w1_s22_ea,vit_s22_t5a >> $O/grain_equal.jsonl
done
for n in 3072 7261 12288 24576 72600; do
  timeout -k 10 120 python tools/vit_tune.py --profile 1400.hmm --n $n --lmin 300 --lmax 500 --longest-first --rounds 2 --variants vit_w1_s22_ea,vit_s22_t5a >> $O/grain_uniform.jsonl
done
timeout -k 10 200 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
