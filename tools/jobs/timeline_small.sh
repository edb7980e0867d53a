set -e
for v in msv_g16_s8_w4_p2_d1 msv_g8_s16_w8_p4_d1 msv_g16_s8_w16_p2_d1; do
  timeout -k 10 120 python tools/wave_timeline.py --config cfg2 --variant $v >> gpurun_out/timeline_cfg2.jsonl 2>/dev/null
done
