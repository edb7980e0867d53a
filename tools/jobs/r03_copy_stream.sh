# One-piece copied host batches put the residues' H2D on the copy stream (offsets + order under it):
# host-path tests, A/B of in-place vs copied page-locked residues by shape, cfg2/cfg3 bench lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_copy_stream
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "pinned or zero_copy or pipeline or cfg2 or small or async or stream or bad_residue or empty" > $O/pytest.log 2>&1
timeout -k 10 400 python tools/zc_wide_ab.py --rounds 3 --modes 1,0 --shapes 100.hmm:10000,200.hmm:10000,400.hmm:10000,100.hmm:100000,1400.hmm:20000,1400.hmm:100000 > $O/ab.jsonl 2> $O/ab.err
timeout -k 10 300 python bench.py --config cfg2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
