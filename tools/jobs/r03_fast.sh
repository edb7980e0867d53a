# Fast blocks (speculative B, branch-free 16-row blocks): GPU suite on the new build, then interleaved
# kernel A/B against the same source built with -DMSV_FASTBLK=0 (ab/base) on cfg2 and small profiles.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_fast
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 4 ab/base/libmsv_hip.so ab/fast/libmsv_hip.so > $O/ab_cfg2.jsonl 2> $O/ab_cfg2.err
for spec in "200.hmm 10000" "200.hmm 100000" "300.hmm 100000" "100.hmm 3000"; do
  set -- $spec
  timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --profile $1 --n $2 --rounds 2 ab/base/libmsv_hip.so ab/fast/libmsv_hip.so >> $O/ab_small.jsonl 2>> $O/ab_small.err
done
timeout -k 10 300 python bench.py --config cfg2 --no-cpu --steps 100 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python tools/bench_reference_programs.py > $O/reference_programs.json 2> $O/reference_programs.err
timeout -k 10 300 python bench.py --config cfg2 --no-cpu --steps 100 --no-launch-events > $O/bench_cfg2_noevents.json 2> $O/bench_cfg2_noevents.err
timeout -k 10 300 python bench.py --config cfg2 --no-cpu --steps 100 > $O/bench_cfg2_b.json 2> $O/bench_cfg2_b.err
