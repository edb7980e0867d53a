# Small profiles at throughput batch sizes: every covering variant (4/8/16/32/64 lanes) at 100k and 1M sequences.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_small
mkdir -p $O
for p in 100.hmm 200.hmm 300.hmm; do
  for n in 100000 1000000; do
    echo "{\"profile\": \"$p\", \"n\": $n}" >> $O/tune_small.jsonl
    timeout -k 10 300 python tools/tune.py --profile $p --n $n --rounds 2 >> $O/tune_small.jsonl
  done
done
