set -e
timeout -k 10 200 python tools/wave_timeline.py --config cfg3 > gpurun_out/timeline_cfg3.jsonl 2>/dev/null
timeout -k 10 200 python tools/wave_timeline.py --config cfg3 --no-order >> gpurun_out/timeline_cfg3.jsonl 2>/dev/null
