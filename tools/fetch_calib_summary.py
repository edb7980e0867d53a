"""FETCH_SIZE calibration factors from a rocprofv3 --pmc FETCH_SIZE pass over tools/micro/fetch_calib.

    python tools/fetch_calib_summary.py <pmc output dir> <known-bytes json printed by fetch_calib>

factor = known bytes read per dispatch / (FETCH_SIZE KiB x 1024), per access pattern; the MSV
kernel's residue stream is the k_ubyte_group pattern (tools/micro/fetch_calib.hip).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, known_path = sys.argv[1], sys.argv[2]
    with open(known_path) as f:
        known = json.loads(f.read().strip().splitlines()[-1])
    per = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = next((k for k in known if k in row.get("Kernel_Name", "")), None)
                if name and row["Counter_Name"] == "FETCH_SIZE":
                    per[name][row["Dispatch_Id"]] += float(row["Counter_Value"])
    res = {}
    for name, disp in per.items():
        kib = sorted(disp.values())
        med = kib[len(kib) // 2]
        res[name] = {"known_bytes": known[name], "fetch_size_kib_per_dispatch": kib,
                     "factor": known[name] / (med * 1024.0)}
    print(json.dumps({"source": "tools/micro/fetch_calib.hip under rocprofv3 --pmc FETCH_SIZE", "kernels": res},
                     indent=1))


if __name__ == "__main__":
    main()
