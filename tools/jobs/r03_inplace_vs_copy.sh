# In-place (zero-copy) vs copied (piece pipeline) page-locked residues by profile size at 100k sequences:
# where the kernel consumes residues faster than the ~25 GB/s in-place read rate, copying wins.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_inplace_vs_copy
mkdir -p $O
timeout -k 10 600 python tools/zc_wide_ab.py --rounds 3 --calls 20 --modes 1,0 --shapes 100.hmm:20000,100.hmm:100000,200.hmm:100000,400.hmm:100000,600.hmm:100000,800.hmm:100000,1001.hmm:100000,1400.hmm:100000 > $O/ab.jsonl 2> $O/ab.err
