"""Cooperative plan vs the plan a batch would otherwise take, by batch size (kernel time on HBM-resident
batches, HIP events on the launch stream; scores compared bitwise).

    python tools/coop_sweep.py --profile 1400.hmm --ns 256,512,1024,2048 [--lmin 300 --lmax 500]

msv_debug_set_coop_max_n(p, 0) turns the cooperative plan off (the latency / mid / main plan runs),
msv_debug_set_coop_max_n(p, huge) sends every batch to it (several sequences per workgroup in turn).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profile", default="1400.hmm")
    ap.add_argument("--ns", default="256,512,1024,2048,4096")
    ap.add_argument("--lmin", type=int, default=300)
    ap.add_argument("--lmax", type=int, default=500)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    lib = _native.lib()
    lib.msv_debug_set_coop_max_n.argtypes = [C.c_void_p, C.c_uint64]
    eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", args.profile)))
    info = eng.describe()
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    for n in (int(x) for x in args.ns.split(",")):
        codes, offsets = random_batch(7, n, args.lmin, args.lmax)
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        order = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        eng.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
        res = {}
        for mode, cap in (("other", 0), ("coop", 1 << 40)) * args.reps:
            assert lib.msv_debug_set_coop_max_n(eng._p, cap) == 0
            s = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(), st.cuda_stream)
            a.record(st)
            eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(), st.cuda_stream)
            b.record(st)
            eng.check(st.cuda_stream)
            res.setdefault(mode, {"ms": [], "scores": None, "variant": eng.variant_for(n)})
            res[mode]["ms"].append(a.elapsed_time(b))
            res[mode]["scores"] = s.cpu().numpy()
        same = bool(np.array_equal(res["coop"]["scores"].view(np.uint32), res["other"]["scores"].view(np.uint32)))
        print(json.dumps({"profile": args.profile, "n": n, "len": [args.lmin, args.lmax],
                          "coop_blocks": info["coop_blocks"], "other_variant": res["other"]["variant"],
                          "coop_variant": res["coop"]["variant"],
                          "other_ms": round(float(np.median(res["other"]["ms"])), 4),
                          "coop_ms": round(float(np.median(res["coop"]["ms"])), 4), "bitwise_equal": same}), flush=True)
    assert lib.msv_debug_set_coop_max_n(eng._p, info["coop_max_n"]) == 0


if __name__ == "__main__":
    main()
