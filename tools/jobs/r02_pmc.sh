# Host-pipeline sweep (same box as the bench line), PMC passes for cfg2 and cfg3.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_pmc
mkdir -p $O
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/host_pipeline_sweep.py --config cfg3 > $O/sweep_cfg3.jsonl 2> $O/sweep_cfg3.err
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 600 bash tools/pmc.sh cfg2 $O/pmc_cfg2 > $O/pmc_cfg2.log 2>&1
timeout -k 10 600 bash tools/pmc.sh cfg3 $O/pmc_cfg3 > $O/pmc_cfg3.log 2>&1
