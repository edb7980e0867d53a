# Round 4 job U: per-wave timeline of cfg2's launch (where its 1.16x over the measured floor goes).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_u
mkdir -p $O
timeout -k 10 200 python tools/wave_timeline.py --config cfg2 > $O/timeline_cfg2.json 2> $O/timeline.err
timeout -k 10 200 python tools/wave_timeline.py --config cfg2 >> $O/timeline_cfg2.json 2>> $O/timeline.err
