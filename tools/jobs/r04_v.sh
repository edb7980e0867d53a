# Round 4 job V: cfg2 dequeue-order dealing A/B (host-built permutation, no kernel change).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_v
mkdir -p $O
timeout -k 10 200 python tools/cfg2_dealing.py --rounds 6 > $O/dealing.jsonl 2> $O/dealing.err
timeout -k 10 200 python tools/cfg2_dealing.py --rounds 6 >> $O/dealing.jsonl 2>> $O/dealing.err
