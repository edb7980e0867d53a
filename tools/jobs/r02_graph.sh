set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02_graph
for c in cfg2 cfg3; do timeout -k 10 200 python tools/graph_probe.py --config $c >> gpurun_out/r02_graph/graph.jsonl 2>> gpurun_out/r02_graph/graph.err; done
