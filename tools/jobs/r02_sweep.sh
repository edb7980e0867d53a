# Kernel rate of all 24 bundled profiles on the cfg3-shaped batch (100k x U[300,500]) and on 10k (cfg2 shape).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_sweep
mkdir -p $O
timeout -k 10 400 python tools/profile_sweep.py --config cfg3 > $O/sweep_cfg3.jsonl
timeout -k 10 300 python tools/profile_sweep.py --config cfg2 --time 20 > $O/sweep_cfg2.jsonl
