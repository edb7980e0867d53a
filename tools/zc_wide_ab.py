"""A/B of the zero-copy twins of residue-block variants: synchronous msv_score_batch calls from page-locked
residues and scores, with the wide-block twin (64-byte superblock requests, msv_debug_set_zero_copy 1)
against the 16-byte blocks of the ordinary variant (mode 2), interleaved over rounds, plus the resident
launch of the same batch for the fraction.  One JSON line per (shape, mode, round).

    python3 tools/zc_wide_ab.py --rounds 3
    python3 tools/zc_wide_ab.py --modes 1,0 --shapes 100.hmm:10000,1400.hmm:100000   (in place vs copied)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [("100.hmm", 10_000, 300, 500, 1), ("100.hmm", 100_000, 300, 500, 2), ("400.hmm", 20_000, 300, 500, 3),
          ("200.hmm", 2_000, 300, 500, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--modes", default="1,2", help="msv_debug_set_zero_copy modes: 1 wide twin, 2 16-B blocks, 0 copied")
    ap.add_argument("--shapes", default="", help="profile:n,... (lengths U[300,500]); default: SHAPES")
    a = ap.parse_args()
    modes = [int(x) for x in a.modes.split(",")]
    shapes = SHAPES if not a.shapes else [(x.split(":")[0], int(x.split(":")[1]), 300, 500, k + 1)
                                          for k, x in enumerate(a.shapes.split(","))]
    import numpy as np
    import torch
    import bench  # noqa: F401  (sets GPU_MAX_HW_QUEUES before HIP starts)
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    L = _native.lib()
    L.msv_debug_set_zero_copy.argtypes = [C.c_void_p, C.c_int]
    for prof, n, lo, hi, seed in shapes:
        e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
        codes, offsets = random_batch(seed, n, lo, hi)
        pc = msv.pinned_empty(codes.size, np.uint8)
        pc[:] = codes
        out = msv.pinned_empty(n, np.float32)
        dev = torch.device("cuda", 0)
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s = torch.empty(n, dtype=torch.float32, device=dev)
        ordt = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.cuda.Stream(dev)

        def resident():
            e.order_longest_first(o.data_ptr(), n, ordt.data_ptr(), st.cuda_stream)
            e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), ordt.data_ptr(), st.cuda_stream)

        ref = None
        for rnd in range(a.rounds):
            for mode in ["resident"] + modes:
                if mode == "resident":
                    for _ in range(5):
                        resident()
                    st.synchronize()
                    t = time.perf_counter()
                    for _ in range(a.calls):
                        resident()
                    st.synchronize()
                    ms = (time.perf_counter() - t) * 1e3 / a.calls
                    got = s.cpu().numpy()
                else:
                    assert L.msv_debug_set_zero_copy(e._p, mode) == 0
                    for _ in range(5):
                        e.score_batch(codes=pc, offsets=offsets, out=out)
                    t = time.perf_counter()
                    for _ in range(a.calls):
                        e.score_batch(codes=pc, offsets=offsets, out=out)
                    ms = (time.perf_counter() - t) * 1e3 / a.calls
                    got = out.copy()
                if ref is None:
                    ref = got
                same = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
                print(json.dumps({"profile": prof, "n": n, "len": [lo, hi], "round": rnd,
                                  "mode": mode if mode == "resident" else {0: "pinned_copy", 1: "pinned_wide", 2: "pinned_16B"}[mode],
                                  "ms_per_call": round(ms, 4), "variant": e.variant_for(n), "bitwise_same": same}),
                      flush=True)
        assert L.msv_debug_set_zero_copy(e._p, 1) == 0
        e.close()


if __name__ == "__main__":
    main()
