#!/bin/bash
# Round 6 job O: model lengths outside the reference's set -- tiny models (LENG 1..99) on every plan, MSV and
# Viterbi, and the first length past the kernel family refused.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_lengths.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
echo ok
