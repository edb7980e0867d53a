# Round 6: short-row MSV kernels with C's update branch-free (two VALU per row off the chain) instead of the
# per-row scalar branch on tr_E_C == tr_E_J: r6base vs r6c, cfg2 kernel + one-wave row time, 200 / 400.hmm batches.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_h
mkdir -p $O
timeout -k 10 200 python -u tools/kernel_ab.py --config cfg2 --rounds 4 abx/r6base/libmsv_hip.so abx/r6c/libmsv_hip.so > $O/ab_cfg2.jsonl 2> $O/ab_cfg2.err
for L in r6base r6c; do MSV_LIB_PATH=$PWD/abx/$L/libmsv_hip.so timeout -k 10 60 python -u tools/cfg2_floor.py > $O/floor_$L.json 2>> $O/floor.err; done
timeout -k 10 200 python -u tools/kernel_ab.py --config cfg2 --profile 400.hmm --rounds 3 abx/r6base/libmsv_hip.so abx/r6c/libmsv_hip.so > $O/ab_400.jsonl 2> $O/ab_400.err
timeout -k 10 200 python -u tools/kernel_ab.py --config cfg2 --profile 200.hmm --rounds 3 abx/r6base/libmsv_hip.so abx/r6c/libmsv_hip.so > $O/ab_200.jsonl 2> $O/ab_200.err
