# A/B: the interleaved asm chunk (max, max, add, max, add, ...) for rows of <= 8 states per lane.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_asm8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py::test_cfg2_full_size_every_score "tests/test_gpu_parity.py::test_homolog_sequences_match_oracle" > $O/pytest.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 4 ab/base/libmsv_hip.so ab/asm8/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --n 2000 --rounds 2 ab/base/libmsv_hip.so ab/asm8/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
