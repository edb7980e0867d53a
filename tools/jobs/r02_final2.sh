# Final pass after the young-wave cutoff: r02_final.sh plus the cfg3 per-wave timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/jobs/r02_final.sh
timeout -k 10 200 python tools/wave_timeline.py --config cfg3 > gpurun_out/final/wave_timeline_cfg3.jsonl
