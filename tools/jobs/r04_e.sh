# Round 4 job E: Viterbi GPU tests (the one-wave-per-SIMD variants added), variant timing on the cfg3 and cfg5
# MSV survivors, and the overlapped one-call path's premises (tools/overlap_probe.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
timeout -k 10 200 python tools/vit_tune.py --config cfg3 --rounds 3 --variants vit_s22_t5,vit_s22_t5a,vit_s22_t7w4,vit_s22_t7w4a,vit_s24_t7w4,vit_s28_t7w4,vit_s38_t7gw4 > $O/vit_tune_cfg3.jsonl 2> $O/vit_tune_cfg3.err
timeout -k 10 300 python tools/vit_tune.py --config cfg5 --rounds 2 > $O/vit_tune_cfg5.jsonl 2> $O/vit_tune_cfg5.err
timeout -k 10 240 python -u tools/overlap_probe.py --reps 30 > $O/overlap_probe.jsonl 2> $O/overlap_probe.err
