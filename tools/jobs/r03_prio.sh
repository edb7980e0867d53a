# Issue priority by length rank for batches that fit the grid once: A/B against -DMSV_RANK_PRIO=0.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_prio
mkdir -p $O
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/prio/libmsv_hip.so > $O/ab.jsonl 2> $O/ab.err
for spec in "200.hmm 10000" "500.hmm 10000" "1400.hmm 3000" "1400.hmm 9000" "900.hmm 9000" "2405.hmm 2000"; do
  set -- $spec
  timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --profile $1 --n $2 --rounds 2 ab/base/libmsv_hip.so ab/prio/libmsv_hip.so >> $O/ab.jsonl 2>> $O/ab.err
done
