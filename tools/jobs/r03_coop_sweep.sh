# Cooperative plan vs the latency / mid / main plan by batch size (where to stop using it).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_coop_sweep
mkdir -p $O
for p in 1400.hmm 400.hmm 100.hmm 1001.hmm 1901.hmm; do
  timeout -k 10 200 python tools/coop_sweep.py --profile $p --ns 64,256,512,1024,2048,4096 >> $O/sweep.jsonl 2>> $O/sweep.err
done
timeout -k 10 200 python tools/coop_sweep.py --profile 2405.hmm --ns 64,256,512,1024 --lmin 1500 --lmax 2500 >> $O/sweep.jsonl 2>> $O/sweep.err
timeout -k 10 200 python tools/coop_sweep.py --profile 1400.hmm --ns 1,3,16,64,256 --lmin 3500 --lmax 3500 >> $O/sweep.jsonl 2>> $O/sweep.err
