# bench.py step composition A/B: each step's sort on the MSV stream (--serial-order) vs on a second
# stream into per-step buffers (default), interleaved, cfg2 and cfg3.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_pipe_order
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu --steps 100 --serial-order > $O/cfg2_serial_$i.json 2> $O/cfg2_serial_$i.err
  timeout -k 10 200 python bench.py --config cfg2 --no-cpu --steps 100 > $O/cfg2_pipe_$i.json 2> $O/cfg2_pipe_$i.err
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg3 --no-cpu --serial-order > $O/cfg3_serial_$i.json 2> $O/cfg3_serial_$i.err
  timeout -k 10 200 python bench.py --config cfg3 --no-cpu > $O/cfg3_pipe_$i.json 2> $O/cfg3_pipe_$i.err
done
