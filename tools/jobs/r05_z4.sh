# Round 5 job Z4: one grid-level exit atomic per workgroup (its last wave, counted in LDS) instead of one per
# wave, in the MSV and Viterbi kernels -- parity first (the GPU suite on the new in-tree build), then
# interleaved A/B vs HEAD: MSV cfg2 / cfg3 (tools/kernel_ab.py), Viterbi cfg2 in place (8,192 waves, 260 with
# work), cfg3, cfg5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_z4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 4 abx/tbase/libmsv_hip.so abx/wgexit/libmsv_hip.so > $O/ab_msv_cfg2.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --rounds 3 abx/tbase/libmsv_hip.so abx/wgexit/libmsv_hip.so > $O/ab_msv_cfg3.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg2 --in-place --variant vit_s2_t7 --rounds 3 abx/tbase/libmsv_hip.so abx/wgexit/libmsv_hip.so > $O/ab_vit_cfg2.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg3 --in-place --variant vit_w1_s22_ea --rounds 3 abx/tbase/libmsv_hip.so abx/wgexit/libmsv_hip.so > $O/ab_vit_cfg3.jsonl
timeout -k 10 300 python tools/vit_ab.py --config cfg5 --in-place --variant vit_w2_s19_gb --rounds 2 abx/tbase/libmsv_hip.so abx/wgexit/libmsv_hip.so > $O/ab_vit_cfg5.jsonl
