# Round 4 job I: Viterbi row-structure A/B at S = 22 (one wave-level branch per row; the next row's first
# chunks requested early; four vs five transition arrays in VGPRs), parity first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
timeout -k 10 300 python tools/vit_tune.py --config cfg3 --longest-first --rounds 4 --variants vit_s22_t5a,vit_s22_t5am,vit_s22_t5amx,vit_s22_t4am,vit_s22_t4amx,vit_s22_t4amx2,vit_s22_t5m,vit_s22_t5 > $O/tune_cfg3.jsonl 2> $O/tune.err
timeout -k 10 300 python tools/vit_tune.py --config cfg4 --longest-first --rounds 2 --variants vit_s22_t5a,vit_s22_t5am,vit_s22_t5amx,vit_s22_t4amx > $O/tune_cfg4.jsonl 2>> $O/tune.err
