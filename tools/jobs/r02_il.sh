# Interleaved static first indices + latency-plan rule (ratio >= 1.3, G=64 BIG cost 1.15, up to 4096*ratio
# sequences): GPU suite, then HEAD (ab/base) vs this build (ab/il) with each build's own plan choice.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_il
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/kernel_ab.py --config cfg2 --rounds 3 ab/base/libmsv_hip.so ab/il/libmsv_hip.so > $O/ab_cfg2.jsonl
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --rounds 3 ab/base/libmsv_hip.so ab/il/libmsv_hip.so > $O/ab_cfg3.jsonl
for n in 3 256 2048 4096 8192; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --profile 1901.hmm --n $n --rounds 2 --warm 3 --time 5 ab/base/libmsv_hip.so ab/il/libmsv_hip.so >> $O/ab_1901.jsonl
done
for n in 2048 8192 12288; do
timeout -k 10 300 python tools/kernel_ab.py --config cfg3 --n $n --rounds 2 --warm 5 --time 10 ab/base/libmsv_hip.so ab/il/libmsv_hip.so >> $O/ab_1400.jsonl
done
