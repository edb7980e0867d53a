"""Sweep of msv_score_batch's copy/compute piece plan (msv_debug_set_pipeline, diagnostics only) on
one config's batch from pinned host memory: mean wall time of `--calls` warm calls per plan, plans
interleaved over `--rounds`, against the HBM-resident single launch (order + kernel).

    python tools/host_pipeline_sweep.py [--config cfg3] [--rounds 3] [--calls 20]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--calls", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bench
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    prof, n, lmin, lmax, seed, _ = bench.CONFIGS[a.config]
    e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
    codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
    pinned = torch.from_numpy(codes).pin_memory().numpy()
    pout = torch.empty(n, dtype=torch.float32).pin_memory().numpy()
    L = _native.lib()
    L.msv_debug_set_pipeline.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32]
    plans = [(0, 2, 1), (4, 2, 2), (5, 2, 2), (6, 2, 2), (8, 2, 2), (6, 3, 2), (8, 3, 2), (3, 2, 2)]
    res = int(offsets[-1])
    want = e.score_batch(codes=codes, offsets=offsets)
    for _ in range(10):  # clock ramp
        e.score_batch(codes=pinned, offsets=offsets)
    for r in range(a.rounds):
        for den, g, ns in plans:
            assert L.msv_debug_set_pipeline(e._p, den, g, ns) == 0
            for _ in range(2):
                e.score_batch(codes=pinned, offsets=offsets, out=pout)
            t = time.perf_counter()
            for _ in range(a.calls):
                out = e.score_batch(codes=pinned, offsets=offsets, out=pout).copy()
            ms = (time.perf_counter() - t) / a.calls * 1e3
            ok = bool(np.array_equal(out.view(np.uint32), want.view(np.uint32)))
            print(json.dumps({"config": a.config, "round": r, "first_den": den, "growth": g, "streams": ns, "ms": round(ms, 4),
                              "M_residues_s": round(res / ms / 1e3, 1), "bitwise_equal": ok}), flush=True)


if __name__ == "__main__":
    main()
