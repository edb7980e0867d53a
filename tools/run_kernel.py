"""Run the MSV kernel alone on a BASELINE config (for rocprofv3 --kernel-trace / --pmc passes).

    python tools/run_kernel.py --config cfg3 --launches 5 [--variant NAME] [--no-order] [--time K]

--time K: after the launches (warm-up), time K more with HIP events on the launch stream and print
one JSON line (kernel ms; A/B of library builds via MSV_LIB_PATH, tools/kernel_ab.py).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--variant", default="")
    ap.add_argument("--no-order", action="store_true")
    ap.add_argument("--time", type=int, default=0)
    ap.add_argument("--profile", default="", help="override the config's profile (e.g. 640.hmm)")
    ap.add_argument("--n", type=int, default=0, help="override the config's sequence count")
    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    prof, n, lmin, lmax, seed, scaling = CONFIGS[args.config]
    prof = args.profile or prof
    n = args.n or n
    eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
    if args.variant:
        eng.set_variant(args.variant)
    # bench.py's rank-0 batch: weak configs seed*1000 + rank, the strong (cfg4) set seed
    codes, offsets = random_batch(seed * 1000 if scaling == "weak" else seed, n, lmin, lmax)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    if not args.no_order:
        eng.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
    op = None if args.no_order else order.data_ptr()
    for _ in range(args.launches):
        eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), op, st.cuda_stream)
    eng.check(st.cuda_stream)
    if args.time:
        import json
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.time)]
        for a, b in ev:
            a.record(st)
            eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), op, st.cuda_stream)
            b.record(st)
        eng.check(st.cuda_stream)
        ms = sorted(a.elapsed_time(b) for a, b in ev)
        print(json.dumps({"config": args.config, "profile": prof, "n": n, "lib": os.environ.get("MSV_LIB_PATH", "in-tree"),
                          "variant": eng.variant_for(n), "kernel_ms_mean": sum(ms) / len(ms),
                          "kernel_ms_median": ms[len(ms) // 2], "kernel_ms_min": ms[0]}), flush=True)
        return
    print(f"{args.config}: {eng.variant_for(n)} x {args.launches} launches, residues={int(offsets[-1])}, "
          f"LENG={eng.model_length - 1}")


if __name__ == "__main__":
    main()
