"""Time every compiled kernel variant that covers a profile on one synthetic batch (one process,
interleaved rounds -- cdna_hip_programming.md §5.4 rule 24) and check they agree bitwise.

    python tools/tune.py --profile 1400.hmm --n 100000 --lmin 300 --lmax 500 [--variants a,b]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profile", default="1400.hmm")
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--lmin", type=int, default=300)
    ap.add_argument("--lmax", type=int, default=500)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", args.profile)))
    leng = eng.model_length - 1
    names = args.variants.split(",") if args.variants else []
    if not names:
        for v in eng.variants():
            if v.startswith("exp"):
                continue
            g, s = int(v.split("_")[1][1:]), int(v.split("_")[2][1:])
            if g * s >= leng and g * s <= leng * 1.35 + 64:
                names.append(v)
    codes, offsets = random_batch(args.seed, args.n, args.lmin, args.lmax)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(args.n, dtype=torch.float32, device=dev)
    order = torch.empty(args.n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    cells = int(offsets[-1]) * leng
    res = {n: [] for n in names}
    ref_scores = None
    for rnd in range(args.rounds):
        for name in names:
            eng.set_variant(name)
            for use_order in (False, True):
                with torch.cuda.stream(st):
                    if use_order:
                        eng.order_longest_first(o.data_ptr(), args.n, order.data_ptr(), st.cuda_stream)
                    op = order.data_ptr() if use_order else None
                    eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), args.n, s.data_ptr(), op,
                                           st.cuda_stream)  # warm
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    ev[0].record(st)
                    for _ in range(args.reps):
                        eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), args.n, s.data_ptr(), op,
                                               st.cuda_stream)
                    ev[1].record(st)
                st.synchronize()
                eng.check(st.cuda_stream)
                ms = ev[0].elapsed_time(ev[1]) / args.reps
                got = s.cpu().numpy()
                if ref_scores is None:
                    ref_scores = got.copy()
                raw = bool(np.array_equal(got.view(np.uint32), ref_scores.view(np.uint32)))
                res[name].append((use_order, ms, raw or name.startswith("exp"), raw))
    out = []
    for name in names:
        for use_order in (False, True):
            t = [ms for (u, ms, _, _) in res[name] if u == use_order]
            same = all(sm for (_, _, sm, _) in res[name])
            raw = all(rw for (_, _, _, rw) in res[name])
            best = min(t)
            out.append({"variant": name, "order": use_order, "ms_min": round(best, 4),
                        "ms_med": round(float(np.median(t)), 4), "Tcell_s": round(cells / best / 1e9, 3),
                        "valu_frac": round(3 * cells / best / 1e9 / 78.64, 4), "bitwise_same": same, "bitwise_same_raw": raw})
    out.sort(key=lambda d: d["ms_min"])
    for d in out:
        print(json.dumps(d))


if __name__ == "__main__":
    main()
