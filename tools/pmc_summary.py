"""Summarise tools/pmc.sh output for the msv_batch_kernel dispatches.

HBM traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB: on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM); our reads are narrow (1-byte residues,
8-byte offsets), for which the factor is uncalibrated, so both the raw and the doubled figure are
reported and the doubled one is used as the (upper-bound) traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, cfg = sys.argv[1], sys.argv[2]
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(out, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "msv_batch_kernel" not in row.get("Kernel_Name", ""):
                    continue
                vals[(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (name, disp), v in vals.items():
        per[name].append(sum(v))
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    dur = []
    for path in glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "msv_batch_kernel" in row["Kernel_Name"]:
                    dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    res = {"config": cfg, "counters_avg_per_dispatch": avg}
    if dur:
        t = sum(dur) / len(dur)
        res["kernel_s_avg"] = t
        if "GRBM_GUI_ACTIVE" in avg:
            res["effective_clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / t / 1e9 if avg["GRBM_GUI_ACTIVE"] > 1e6 else None
    if "FETCH_SIZE" in avg:
        res["fetch_kib_raw"] = avg["FETCH_SIZE"]
        res["write_kib"] = avg.get("WRITE_SIZE")
        res["hbm_bytes_per_launch"] = int((2 * avg["FETCH_SIZE"] + avg.get("WRITE_SIZE", 0)) * 1024)
    if "SQ_ACTIVE_INST_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # VALUBusy as rocprofv3 defines it: SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE
        res["valu_busy_pct"] = 100 * avg["SQ_ACTIVE_INST_VALU"] / 256 / (avg["GRBM_GUI_ACTIVE"] / 8)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
