# Round 6: every compiled MSV variant that covers 100.hmm re-timed on cfg2's shape (10,000 x U[300,500], seed
# 1000 = bench.py's rank-0 batch), with and without the longest-first order, at the final kernels.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_k
mkdir -p $O
timeout -k 10 300 python -u tools/tune.py --profile 100.hmm --n 10000 --lmin 300 --lmax 500 --seed 1000 --rounds 3 > $O/tune_cfg2.jsonl 2> $O/tune_cfg2.err
