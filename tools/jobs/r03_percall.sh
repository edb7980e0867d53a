# Timeline of the reference's per-sequence call pattern (parallel_run_on_sequence, 1400.hmm x random_FASTA,
# pageable): kernel + copy trace of single calls.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_percall
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --per-sequence 1400.hmm --calls 30 --mark 6 > $O/calls.txt 2> $O/calls.err
python3 tools/pipeline_timeline.py $(find $O/trace -name '*kernel_trace.csv') $(find $O/trace -name '*memory_copy_trace.csv') > $O/timeline.txt 2>&1
