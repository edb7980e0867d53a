# Round 5 job K: (1) W = 1 team kernel vs vit_kernel's S = 20/22 picks (job J's steps), (2) VERDICT r04 item 7:
# the MSV score store as a non-temporal store -- WRITE_SIZE per launch and kernel time against HEAD (cfg3).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/jobs/r05_j.sh
O=gpurun_out/r05_k
mkdir -p $O
for b in head ntstore; do
  MSV_LIB_PATH=$PWD/abx/$b/libmsv_hip.so timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/ws_$b/pmc1 -o run -- python3 tools/run_kernel.py --config cfg3 --launches 3 > $O/ws_$b.log 2>&1
  MSV_LIB_PATH=$PWD/abx/$b/libmsv_hip.so timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ws_$b/pmc2 -o run -- python3 tools/run_kernel.py --config cfg3 --launches 3 >> $O/ws_$b.log 2>&1
  python3 tools/pmc_summary.py $O/ws_$b cfg3 > $O/ws_$b.json || true
done
timeout -k 10 400 python tools/kernel_ab.py --config cfg3 --rounds 4 abx/head/libmsv_hip.so abx/ntstore/libmsv_hip.so > $O/ab_ntstore_cfg3.jsonl
# the E identity on small rows (MSV_IDENTITY_E build) -- parity against HEAD's scores
# (cfg2 batch + homologs, whose J passes N) and the interleaved kernel A/B on cfg2
for b in head ident; do
  MSV_LIB_PATH=$PWD/abx/$b/libmsv_hip.so timeout -k 10 120 python tools/lib_scores.py --config cfg2 --out $O/scores_$b.npy
done
python3 -c "import numpy as np; a=np.load('$O/scores_head.npy'); b=np.load('$O/scores_ident.npy'); print('ident bitwise_equal', bool((a==b).all()), len(a))" > $O/ident_parity.txt
timeout -k 10 400 python tools/kernel_ab.py --config cfg2 --rounds 4 abx/head/libmsv_hip.so abx/ident/libmsv_hip.so > $O/ab_ident_cfg2.jsonl
