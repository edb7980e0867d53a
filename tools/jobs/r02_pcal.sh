set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02_pcal
timeout -k 10 300 python tools/pvalue_calibration.py > gpurun_out/r02_pcal/calib.jsonl
