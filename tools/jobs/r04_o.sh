# Round 4 job O: Viterbi parity with the one-move wave_shr lane shift, then A/B against the previous build
# (ab/vbase) on the cfg3 / cfg5 / cfg4 survivors, alternating processes (MSV_LIB_PATH).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_viterbi.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_vit.log 2>&1
for r in 1 2 3; do
  for lib in ab/vbase/libmsv_hip.so hmm_fasta_viterbi_amd/lib/libmsv_hip.so; do
    MSV_LIB_PATH=$lib timeout -k 10 200 python tools/vit_tune.py --config cfg3 --longest-first --rounds 1 --variants vit_s22_t5a,vit_s22_t5 | sed "s#^{#{\"lib\": \"$lib\", #" >> $O/ab_cfg3.jsonl
    MSV_LIB_PATH=$lib timeout -k 10 200 python tools/vit_tune.py --config cfg5 --longest-first --rounds 1 --reps 3 --variants vit_s38_t7gw4 | sed "s#^{#{\"lib\": \"$lib\", #" >> $O/ab_cfg5.jsonl
  done
done
for lib in ab/vbase/libmsv_hip.so hmm_fasta_viterbi_amd/lib/libmsv_hip.so; do
  MSV_LIB_PATH=$lib timeout -k 10 300 python tools/vit_tune.py --config cfg4 --longest-first --rounds 1 --reps 3 --variants vit_s22_t5a | sed "s#^{#{\"lib\": \"$lib\", #" >> $O/ab_cfg4.jsonl
done
