# Order kernels after the fused scan: GPU suite, smoke, bench cfg3 + its rocprofv3 trace, bench cfg2 + trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/jobs/r02_verify.sh
O=gpurun_out/r02_verify
timeout -k 10 240 python bench.py --config cfg2 --no-cpu --steps 50 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --config cfg2 --no-cpu --steps 50 > $O/bench_cfg2_prof.json 2>&1
