# Small host calls staged (residues in the offsets' H2D, pageable scores through pinned staging): the GPU
# suite, the reference's benchmark programs, and the per-sequence call timeline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_smallcall
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/bench_reference_programs.py > $O/reference_programs.json 2> $O/reference_programs.err
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --per-sequence 1400.hmm --calls 30 --mark 6 > $O/calls.txt 2> $O/calls.err
python3 tools/pipeline_timeline.py $(find $O/trace -name '*kernel_trace.csv') $(find $O/trace -name '*memory_copy_trace.csv') > $O/timeline.txt 2>&1
