# Zero-copy probe: residues read by the kernel from pinned host memory vs resident in HBM.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02_zc
mkdir -p $O
timeout -k 10 120 python tools/zero_copy_probe.py --config cfg2 > $O/zc.jsonl
timeout -k 10 200 python tools/zero_copy_probe.py --config cfg3 >> $O/zc.jsonl
timeout -k 10 200 python tools/zero_copy_probe.py --config cfg3 --offsets-host >> $O/zc.jsonl
timeout -k 10 200 python tools/zero_copy_probe.py --config cfg3 --variant msv_g32_s44_w16_p2_d1 >> $O/zc.jsonl
