"""Print the last calls of tools/host_pipeline_trace.py as a timeline: every kernel dispatch and
memory copy between consecutive host gaps, times relative to the call's first event (us)."""
import csv
import sys


def main():
    kt, mt = sys.argv[1], sys.argv[2]
    ev = []
    for r in csv.DictReader(open(kt)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
    for r in csv.DictReader(open(mt)):
        name = r.get("Direction") or r.get("Operation") or "copy"
        size = r.get("Size", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"C {name} {size}"))
    ev.sort()
    # calls are separated by >= 0.5 ms of idle GPU time; print the last 3 groups
    groups, cur, end = [], [], 0
    for e in ev:
        if cur and e[0] - end > 500_000:
            groups.append(cur)
            cur = []
        cur.append(e)
        end = max(end, e[1])
    groups.append(cur)
    for g in groups[-3:]:
        t0 = g[0][0]
        last = max(e[1] for e in g)
        print(f"--- call: {(last - t0) / 1e3:.1f} us, {len(g)} events")
        for s, e, name in g:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}")


if __name__ == "__main__":
    main()
