# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks, gloo collectives, both on cuda:0.
set -e
export MSV_BENCH_BACKEND=gloo MSV_BENCH_ONE_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/rehearse_2rank.json 2> gpurun_out/rehearse_2rank.err
