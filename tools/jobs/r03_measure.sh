# Round-3 measurement pass at HEAD: bench lines for cfg2/3/4/5 (cfg3 = the driver's default command),
# rocprofv3 kernel-trace summaries + exact-variant windows of the same commands, PMC passes for every
# config through tools/pmc.sh (name-checked, calibrated), the cfg5 per-wave timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_measure
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/r02/libmsv_hip.so ab/r03/libmsv_hip.so > $O/ab_r02_r03_cfg3.jsonl 2> $O/ab_cfg3.err
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/r02/libmsv_hip.so ab/r03/libmsv_hip.so > $O/ab_r02_r03_cfg2.jsonl 2> $O/ab_cfg2.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py --config cfg5 --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 400 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
timeout -k 10 300 python tools/bench_reference_programs.py > $O/reference_programs.json 2> $O/reference_programs.err
