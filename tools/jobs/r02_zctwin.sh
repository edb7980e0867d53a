# Zero-copy twins: GPU suite, zero-copy probe (cfg3, cfg4-size), bench cfg3 host paths.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_zctwin
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3_b.json 2> $O/bench_cfg3_b.err
timeout -k 10 400 python bench.py --no-cpu --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
