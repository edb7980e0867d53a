set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "fasta" > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_ingest.py > gpurun_out/ingest.json 2> gpurun_out/ingest.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ingest_prof -o run -- python3 tools/bench_ingest.py --n 300000 > gpurun_out/ingest_prof.json 2>&1
