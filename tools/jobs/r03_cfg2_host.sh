# cfg2 host call (msv_score_batch from page-locked residues): kernel + copy trace of single calls.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_cfg2_host
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 tools/host_pipeline_trace.py --config cfg2 --calls 30 --mark 3 > $O/calls.txt 2> $O/calls.err
python3 tools/pipeline_timeline.py $(find $O/trace -name '*kernel_trace.csv') $(find $O/trace -name '*memory_copy_trace.csv') > $O/timeline.txt 2>&1
timeout -k 10 200 python3 tools/host_pipeline_trace.py --config cfg2 --calls 30 --mark 3 > $O/calls_noprof.txt 2>&1
