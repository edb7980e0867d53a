# A/B: per-row event check marked unlikely for rows of <= 40 states per lane (HEAD layout: two taken
# branches per row on the common path).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_unlikely
mkdir -p $O
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/new/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --rounds 2 ab/base/libmsv_hip.so ab/new/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
timeout -k 10 300 python tools/kernel_ab.py --config cfg5 --rounds 2 --warm 3 --time 5 ab/base/libmsv_hip.so ab/new/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
for p in 400.hmm 600.hmm 200.hmm 800.hmm; do
  timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --profile $p --n 100000 --rounds 2 ab/base/libmsv_hip.so ab/new/libmsv_hip.so >> $O/ab.jsonl 2>> $O/err.txt
done
