"""Summarise tools/pmc.sh output for the msv_batch_kernel dispatches.

HBM traffic per launch = factor * FETCH_SIZE + WRITE_SIZE.  On gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM) and is uncalibrated for other widths; the
MSV kernel's reads are dominated (~94% of its bytes) by the residue stream, 1-byte loads that 16
lanes issue to one address, so `factor` is the one MEASURED for exactly that pattern by
tools/micro/fetch_calib.hip (profiles/r02_fetch_calib.json, kernel k_ubyte_group); without that
file the guide's factor 2 is used and the figure is flagged uncalibrated.

VALU issue busy = SQ_INSTS_VALU x 2 cycles (a wave64 VALU instruction occupies a SIMD32 for 2
cycles) / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8): GRBM_GUI_ACTIVE is summed over the 8 XCDs (its
per-XCD value over the kernel time gives the clock).  This counts issue slots of full-rate
instructions; v_max/v_max3 occupy about twice that (tools/micro/valu_rate.hip).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, cfg = sys.argv[1], sys.argv[2]
    kname = sys.argv[3] if len(sys.argv) > 3 else "msv_batch_kernel"  # e.g. vit_kernel (tools/run_vit.py)
    vals = defaultdict(list)
    names = set()
    for path in glob.glob(os.path.join(out, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kname not in row.get("Kernel_Name", ""):
                    continue
                names.add(row["Kernel_Name"])
                # per pass: Dispatch_Id restarts in every rocprofv3 run
                vals[(row["Counter_Name"], path, row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    # Every pass must have measured ONE kernel (tools/run_kernel.py launches the resident variant only);
    # bench.py publishes roofline.traffic only when this name is the kernel its timed steps run.
    if len(names) != 1:
        sys.exit(f"pmc_summary: expected one {kname} instantiation, found {sorted(names)}")
    per = defaultdict(list)
    for (name, _path, _disp), v in vals.items():
        per[name].append(sum(v))
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    dur = []
    for path in glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Kernel_Name"] in names:
                    dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    res = {"config": cfg, "kernel": next(iter(names)), "counters_avg_per_dispatch": avg}
    if dur:
        t = sum(dur) / len(dur)
        res["kernel_s_avg"] = t
        if "GRBM_GUI_ACTIVE" in avg:
            res["effective_clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / t / 1e9 if avg["GRBM_GUI_ACTIVE"] > 1e6 else None
    if "FETCH_SIZE" in avg:
        factor, calibrated = 2.0, False
        cal = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r02_fetch_calib.json")
        if os.path.exists(cal):
            with open(cal) as f:
                factor = json.load(f)["kernels"]["k_ubyte_group"]["factor"]
            calibrated = True
        res["fetch_kib_raw"] = avg["FETCH_SIZE"]
        res["write_kib"] = avg.get("WRITE_SIZE")
        res["fetch_factor"] = factor
        res["fetch_factor_calibrated"] = calibrated
        res["hbm_bytes_per_launch"] = int((factor * avg["FETCH_SIZE"] + avg.get("WRITE_SIZE", 0)) * 1024)
    if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        res["valu_issue_busy_pct"] = 100 * avg["SQ_INSTS_VALU"] * 2 / 1024 / (avg["GRBM_GUI_ACTIVE"] / 8)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
