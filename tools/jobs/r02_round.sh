# Round-2 GPU pass: parity suite (incl. full-size cfg4/cfg5), bench cfg3 + cfg4 + cfg2, FETCH_SIZE
# calibration of the narrow-read patterns, a 2-rank rehearsal of bench.py --config cfg4.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_round
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python bench.py --config cfg4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
timeout -k 10 300 python bench.py --config cfg2 --no-cpu > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- ./tools/micro/fetch_calib > $O/fetch_known.json 2> $O/fetch.err
python3 tools/fetch_calib_summary.py $O/fetch $O/fetch_known.json > $O/fetch_calib.json
export MSV_BENCH_BACKEND=gloo MSV_BENCH_ONE_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --config cfg4 --steps 3 --warmup 1 --no-cpu > $O/rehearse_cfg4_2rank.json 2> $O/rehearse_cfg4_2rank.err
