# In-place policy by model size: host-path tests, then the GPU suite in full, bench cfg2/cfg3.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_policy
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python tools/zc_wide_ab.py --rounds 2 --calls 20 --modes 1 --shapes 100.hmm:100000,200.hmm:100000,400.hmm:100000 > $O/ab_policy.jsonl 2> $O/ab.err
