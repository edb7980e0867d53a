"""Average kernel duration over bench.py's timed window from a rocprofv3 --kernel-trace CSV.

    python tools/rocprof_window.py <run_kernel_trace.csv> --kernel msv_batch_kernel --skip W --take K

bench.py launches the MSV kernel W (warmup) + K (timed) times, then once more per informational
path (host-buffer, pinned).  rocprofv3 --stats averages all of them, including the launches while
the GPU clock is still ramping (first ~10) and after the CPU-side pauses; this prints the average of
dispatches W+1 .. W+K, the ones bench.py's HIP events time.
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="msv_batch_kernel")
    ap.add_argument("--skip", type=int, default=12)
    ap.add_argument("--take", type=int, default=20)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    w = d[a.skip:a.skip + a.take]
    print(json.dumps({"kernel": rows[0]["Kernel_Name"] if rows else a.kernel, "dispatches": len(d),
                      "window": [a.skip, a.skip + len(w)], "avg_us": round(sum(w) / max(len(w), 1), 1),
                      "min_us": round(min(w), 1) if w else None, "max_us": round(max(w), 1) if w else None,
                      "all_avg_us": round(sum(d) / max(len(d), 1), 1), "all_us": [round(x) for x in d]}))


if __name__ == "__main__":
    main()
