# Round 6: the Viterbi kernels against the explicitly enumerated best state path on tiny models.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_i
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_viterbi_paths.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_paths.log 2>&1
