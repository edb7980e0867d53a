"""Average kernel duration over bench.py's timed window from a rocprofv3 --kernel-trace CSV.

    python tools/rocprof_window.py <run_kernel_trace.csv> --kernel msv_batch_kernel --last K
    python tools/rocprof_window.py <run_kernel_trace.csv> --skip W --take K

bench.py (round 2) launches the MSV kernel for its informational host paths first, then W warmup
and K timed steps, and nothing after them (with --no-cpu), so its timed window is the LAST K
dispatches.  rocprofv3 --stats averages all dispatches, including the host-path pieces and the
launches while the GPU clock ramps; this prints the average over the window bench.py's HIP events time.
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
    ap.add_argument("--last", type=int, default=0, help="window = the last N dispatches (overrides --skip/--take)")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if a.last:
        a.skip, a.take = max(0, len(d) - a.last), a.last
    w = d[a.skip:a.skip + a.take]
    print(json.dumps({"kernel": rows[0]["Kernel_Name"] if rows else a.kernel, "dispatches": len(d),
                      "window": [a.skip, a.skip + len(w)], "avg_us": round(sum(w) / max(len(w), 1), 1),
                      "min_us": round(min(w), 1) if w else None, "max_us": round(max(w), 1) if w else None,
                      "all_avg_us": round(sum(d) / max(len(d), 1), 1), "all_us": [round(x) for x in d]}))


if __name__ == "__main__":
    main()
