# GPU suite after the late next-index fetch; bench cfg3 + cfg5 (with the two-stream information);
# 2-rank rehearsal of bench.py (cfg3 weak, cfg4 strong) with gloo on the one GPU.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_check3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --no-cpu > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --no-cpu --config cfg5 --steps 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
export MSV_BENCH_BACKEND=gloo MSV_BENCH_ONE_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > $O/rehearse_cfg3_2rank.json 2> $O/rehearse_cfg3_2rank.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 2 --config cfg4 --steps 3 --warmup 1 --no-cpu > $O/rehearse_cfg4_2rank.json 2> $O/rehearse_cfg4_2rank.err
