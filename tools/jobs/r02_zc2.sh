# Zero-copy host path: GPU suite, bench lines (host figures: zero-copy, copy pipeline, streamed) for
# cfg3/cfg4/cfg5/cfg2, zero-copy probe on cfg5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_zc2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --no-cpu --config cfg4 --steps 5 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
timeout -k 10 300 python bench.py --no-cpu --config cfg5 --steps 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 300 python bench.py --no-cpu --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 200 python tools/zero_copy_probe.py --config cfg5 --time 4 > $O/zc_cfg5.jsonl
