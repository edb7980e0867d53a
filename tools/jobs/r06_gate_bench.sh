#!/bin/bash
# Record the bench-config MSV speeds into a copy of the speed table, then run the whole gate against it.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp tests/golden/speed_table.json gpurun_out/speed_table.json
SPEED_GATE_RECORD=gpurun_out/speed_table.json timeout -k 10 300 python -u -m pytest tests/test_speed_gate.py -k bench_configs -x -v -s --timeout 240 --timeout-method thread > gpurun_out/gate_record.log 2>&1
cp gpurun_out/speed_table.json tests/golden/speed_table.json
timeout -k 10 300 python -u -m pytest tests/test_speed_gate.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/gate_check.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_speed_gate.py -k bench_configs -x -v -s --timeout 240 --timeout-method thread > gpurun_out/gate_check2.log 2>&1
echo done
