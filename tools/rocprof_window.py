"""Average kernel duration over bench.py's timed window from a rocprofv3 --kernel-trace CSV.

    python tools/rocprof_window.py <run_kernel_trace.csv> --variant msv_g16_s88_w16_p2_d1 --last K
    python tools/rocprof_window.py <run_kernel_trace.csv> --kernel 'msv_batch_kernel<16, 88, ...>' --skip W --take K

Dispatches are filtered on ONE exact kernel: --variant maps the library's variant name (bench.py's
`config.kernel_variant`) to its HBM-resident instantiation (hmm_fasta_viterbi_amd.kernel_names), so the
zero-copy twins that bench.py's informational host paths launch (`..., 2>`) are never averaged in or
used as the label.  A --kernel substring that matches more than one distinct kernel is an error.

bench.py launches the MSV kernel for its informational host paths first, then W warmup and K timed
steps, and nothing after them (with --no-cpu), so its timed window is the LAST K dispatches of the
resident kernel.  rocprofv3 --stats averages all dispatches, including the host-path pieces and the
launches while the GPU clock ramps; this prints the average over the window bench.py's HIP events time.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    g = ap.add_mutually_exclusive_group(required=True)
    g.add_argument("--variant", help="library variant name; window over its resident instantiation")
    g.add_argument("--kernel", help="substring of exactly one kernel name")
    ap.add_argument("--zero-copy", action="store_true", help="with --variant: the zero-copy twin instead")
    ap.add_argument("--skip", type=int, default=12)
    ap.add_argument("--take", type=int, default=20)
    ap.add_argument("--last", type=int, default=0, help="window = the last N dispatches (overrides --skip/--take)")
    a = ap.parse_args()
    if a.variant:
        from hmm_fasta_viterbi_amd.kernel_names import kernel_symbol
        want = kernel_symbol(a.variant, zero_copy=a.zero_copy)
    else:
        want = a.kernel
    rows = [r for r in csv.DictReader(open(a.trace)) if want in r["Kernel_Name"]]
    names = sorted({r["Kernel_Name"] for r in rows})
    if len(names) != 1:
        sys.exit(f"rocprof_window: {want!r} matches {len(names)} kernels: {names}")
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if a.last:
        a.skip, a.take = max(0, len(d) - a.last), a.last
    w = d[a.skip:a.skip + a.take]
    print(json.dumps({"kernel": names[0], "variant": a.variant, "dispatches": len(d),
                      "window": [a.skip, a.skip + len(w)], "avg_us": round(sum(w) / max(len(w), 1), 1),
                      "min_us": round(min(w), 1) if w else None, "max_us": round(max(w), 1) if w else None,
                      "all_avg_us": round(sum(d) / max(len(d), 1), 1), "all_us": [round(x) for x in d]}))


if __name__ == "__main__":
    main()
