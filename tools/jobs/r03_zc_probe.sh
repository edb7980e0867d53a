# Zero-copy follow-up: host allocation flags vs in-place read rate (cfg2), wide-twin A/B after restricting
# the twins to PF <= 2 variants, zero-copy parity tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_zc_probe
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "zero_copy or pinned" > $O/pytest_zc.log 2>&1
timeout -k 10 200 python tools/zc_host_memory_probe.py > $O/host_memory.jsonl 2> $O/host_memory.err
timeout -k 10 300 python tools/zc_wide_ab.py --rounds 2 > $O/ab.jsonl 2> $O/ab.err
