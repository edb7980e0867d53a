#!/bin/bash
# Round 6 job M: the multi-rank bench path at HEAD, rehearsed on one GPU (gloo collectives on host tensors,
# every rank on cuda:0): cfg3 (weak) and cfg4 (strong, gather) at 2 ranks, cfg4 at 4 ranks.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_m
mkdir -p $O
export MSV_BENCH_BACKEND=gloo MSV_BENCH_ONE_DEVICE=1
timeout -k 10 300 python bench.py --gpus 2 --config cfg3 --steps 10 --warmup 5 > $O/cfg3_2rank.json 2> $O/cfg3_2rank.err
timeout -k 10 300 python bench.py --gpus 2 --config cfg4 --steps 5 --warmup 3 > $O/cfg4_2rank.json 2> $O/cfg4_2rank.err
timeout -k 10 300 python bench.py --gpus 4 --config cfg4 --steps 5 --warmup 3 > $O/cfg4_4rank.json 2> $O/cfg4_4rank.err
echo ok
