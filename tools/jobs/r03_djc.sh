# Delayed J check (double-buffered <= 8-state rows): parity on the plans that run it, then kernel A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_djc
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py::test_cfg2_full_size_every_score "tests/test_gpu_parity.py::test_homolog_sequences_match_oracle" tests/test_gpu_parity.py::test_narrow_plan_full_batches_match "tests/test_gpu_parity.py::test_seeded_golden_edge_lengths" tests/test_gpu_parity.py::test_distinct_tr_E_C_and_tr_E_J "tests/test_gpu_parity.py::test_latency_plan_small_batches_match_main_plan" > $O/pytest.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 4 ab/base/libmsv_hip.so ab/djc/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --n 2000 --rounds 2 ab/base/libmsv_hip.so ab/djc/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
