# Round 4 job D: the overlapped one-call path's two premises (tools/overlap_probe.py: in-place reads under
# a concurrent SDMA copy; stream-ordered flag latency under a full grid).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_d
mkdir -p $O
timeout -k 10 240 python -u tools/overlap_probe.py --reps 30 > $O/overlap_probe.jsonl 2> $O/overlap_probe.err
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --rounds 3 > $O/vit_tune_cfg5.jsonl 2> $O/vit_tune_cfg5.err
