"""Probe: how fast the kernel reads page-locked residues in place depending on the host allocation's
flags (hipHostMalloc default / coherent / non-coherent / write-combined / uncached), on cfg2's batch
(100.hmm x 10k, 4 MB): mean synchronous msv_score_batch call and an SDMA H2D copy of the same bytes.
Scores must equal the resident launch bitwise.  One JSON line per flag set.

    python3 tools/zc_host_memory_probe.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FLAGS = {"default": 0x0, "portable": 0x1, "coherent": 0x40000000, "noncoherent": 0x80000000,
         "writecombined": 0x4 | 0x2, "uncached": 0x10000000}


def main():
    import numpy as np
    import torch
    import bench  # noqa: F401  (sets GPU_MAX_HW_QUEUES before HIP starts)
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    hip = C.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipHostFree.argtypes = [C.c_void_p]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipDeviceSynchronize.argtypes = []
    e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", "100.hmm")))
    codes, offsets = random_batch(1, 10_000, 300, 500)
    n = len(offsets) - 1
    want = e.score_batch(codes=codes, offsets=offsets)
    d = torch.empty(codes.size, dtype=torch.uint8, device="cuda")
    for name, fl in FLAGS.items():
        p = C.c_void_p()
        rc = hip.hipHostMalloc(C.byref(p), codes.size, fl)
        if rc != 0:
            print(json.dumps({"flags": name, "error": rc}), flush=True)
            continue
        buf = np.ctypeslib.as_array((C.c_uint8 * codes.size).from_address(p.value))
        buf[:] = codes
        for _ in range(5):
            got = e.score_batch(codes=buf, offsets=offsets)
        t = time.perf_counter()
        for _ in range(50):
            got = e.score_batch(codes=buf, offsets=offsets)
        call_ms = (time.perf_counter() - t) * 1e3 / 50
        hip.hipDeviceSynchronize()
        t = time.perf_counter()
        for _ in range(20):
            hip.hipMemcpy(C.c_void_p(d.data_ptr()), p, codes.size, 1)  # hipMemcpyHostToDevice
        h2d_ms = (time.perf_counter() - t) * 1e3 / 20
        print(json.dumps({"flags": name, "value": fl, "call_ms": round(call_ms, 4), "h2d_ms": round(h2d_ms, 4),
                          "h2d_GBps": round(codes.size / h2d_ms / 1e6, 1), "variant": e.variant_for(n),
                          "bitwise_equal": bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))}),
              flush=True)
        del buf, got
        hip.hipHostFree(p)
    e.close()


if __name__ == "__main__":
    main()
