"""Probe for the overlapped one-call path: an SDMA copy of a small model's batch
running under the kernel that reads the same residues in place, each chunk handed over by a
stream-ordered flag.  Two premises decide whether that path can beat cfg2's one-call fraction (~0.5):

  A. link sharing -- does the kernel's in-place read rate (~25 GB/s) survive an SDMA H2D
     copy (~50 GB/s) running at the same time, i.e. do the two add up?  cfg2's batch (100.hmm x 10k,
     4 MB, bench seed 1000) through msv_score_batch from page-locked memory (the in-place path), alone
     and with a 16 MB H2D copy of other pinned bytes in flight on another stream for the whole call;
     the copy alone and under the call.
  B. flag latency under a full grid -- when does a stream-ordered flag land while a persistent MSV grid
     (1400.hmm x 100k resident, ~2.8 ms) holds every CU?  hipStreamWriteValue32 into a page-locked word
     (polled by the host) and a 4-byte SDMA H2D copy followed by an event, each on its own stream,
     issued right after the grid; landing times relative to the grid's own end event.

One JSON line per measurement; scores of every call are checked bitwise against the resident launch.

    python3 tools/overlap_probe.py [--reps 30]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench  # noqa: F401  (sets GPU_MAX_HW_QUEUES before HIP starts)
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    hip = C.CDLL("libamdhip64.so")
    vp = C.c_void_p
    hip.hipHostMalloc.argtypes = [C.POINTER(vp), C.c_size_t, C.c_uint]
    hip.hipHostFree.argtypes = [vp]
    hip.hipMemcpyAsync.argtypes = [vp, vp, C.c_size_t, C.c_int, vp]
    hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(vp), C.c_uint]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipEventCreate.argtypes = [C.POINTER(vp)]
    hip.hipEventRecord.argtypes = [vp, vp]
    hip.hipEventQuery.argtypes = [vp]
    hip.hipEventSynchronize.argtypes = [vp]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), vp, vp]
    hip.hipStreamWriteValue32.argtypes = [vp, vp, C.c_uint32, C.c_uint]
    hip.hipDeviceSynchronize.argtypes = []

    def stream():
        s = vp()
        assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0  # non-blocking
        return s

    def event():
        e = vp()
        assert hip.hipEventCreate(C.byref(e)) == 0
        return e

    def pinned(nbytes):
        p = vp()
        assert hip.hipHostMalloc(C.byref(p), nbytes, 0) == 0
        return p, np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p.value))

    def elapsed(e0, e1):
        t = C.c_float()
        assert hip.hipEventElapsedTime(C.byref(t), e0, e1) == 0
        return float(t.value)

    def emit(d):
        print(json.dumps(d), flush=True)

    # ---- A. link sharing --------------------------------------------------------------------------
    e100 = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", "100.hmm")))
    codes, offsets = random_batch(1000, 10_000, 300, 500)
    want = e100.score_batch(codes=codes, offsets=offsets)
    pres, buf = pinned(codes.size)
    buf[:] = codes
    big = 16 << 20
    psrc, _ = pinned(big)
    dst = torch.empty(big, dtype=torch.uint8, device="cuda")
    sc = stream()
    c0, c1 = event(), event()

    def copy_alone():
        hip.hipEventRecord(c0, sc)
        hip.hipMemcpyAsync(vp(dst.data_ptr()), psrc, big, 1, sc)
        hip.hipEventRecord(c1, sc)
        hip.hipStreamSynchronize(sc)
        return elapsed(c0, c1)

    def call_alone():
        t = time.perf_counter()
        got = e100.score_batch(codes=buf, offsets=offsets)
        ms = (time.perf_counter() - t) * 1e3
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        return ms

    def call_under_copy():
        hip.hipEventRecord(c0, sc)
        hip.hipMemcpyAsync(vp(dst.data_ptr()), psrc, big, 1, sc)
        hip.hipEventRecord(c1, sc)
        time.sleep(20e-6)  # let the copy start first
        ms = call_alone()
        hip.hipStreamSynchronize(sc)
        return ms, elapsed(c0, c1)

    for _ in range(5):
        copy_alone(), call_alone(), call_under_copy()
    alone_call, alone_copy, both_call, both_copy = [], [], [], []
    for _ in range(a.reps):  # interleaved
        alone_call.append(call_alone())
        alone_copy.append(copy_alone())
        x, y = call_under_copy()
        both_call.append(x)
        both_copy.append(y)
    med = lambda v: round(float(np.median(v)), 4)  # noqa: E731
    emit({"probe": "A_link_sharing", "batch": "cfg2 (100.hmm x 10k, 4 MB, seed 1000)", "copy_bytes": big,
          "in_place_call_ms_alone": med(alone_call), "in_place_call_ms_under_copy": med(both_call),
          "copy_ms_alone": med(alone_copy), "copy_ms_under_call": med(both_copy),
          "copy_GBps_alone": round(big / med(alone_copy) / 1e6, 1),
          "in_place_call_slowdown": round(med(both_call) / med(alone_call), 3), "reps": a.reps,
          "resident_variant": e100.variant_for(len(offsets) - 1), "bitwise_equal": True})
    hip.hipHostFree(pres)
    hip.hipHostFree(psrc)
    del buf, dst

    # ---- B. flag latency under a full grid -------------------------------------------------------
    e1400 = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", "1400.hmm")))
    codes, offsets = random_batch(3, 100_000, 300, 500)
    n = len(offsets) - 1
    r = torch.from_numpy(codes).cuda()
    o = torch.from_numpy(offsets.view(np.int64)).cuda()
    s = torch.empty(n, dtype=torch.float32, device="cuda")
    order = torch.empty(n, dtype=torch.int32, device="cuda")
    sk, sw, sd = stream(), stream(), stream()
    pflag, flag = pinned(64)
    pword, _ = pinned(64)
    dword = torch.zeros(16, dtype=torch.int32, device="cuda")
    k0, k1, d1 = event(), event(), event()
    e1400.order_longest_first(o.data_ptr(), n, order.data_ptr(), sk.value)
    hip.hipStreamSynchronize(sk)
    rows = []
    for rep in range(8):
        flag[:] = 0
        hip.hipDeviceSynchronize()
        hip.hipEventRecord(k0, sk)
        e1400.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(), sk.value)
        hip.hipEventRecord(k1, sk)
        t0 = time.perf_counter()
        time.sleep(200e-6)  # the grid is running by now
        t_issue = time.perf_counter()
        rc = hip.hipStreamWriteValue32(sw, pflag, rep + 1, 0)
        hip.hipMemcpyAsync(vp(dword.data_ptr()), pword, 4, 1, sd)
        hip.hipEventRecord(d1, sd)
        t_flag = t_copy = t_end = None
        while t_end is None or t_flag is None or t_copy is None:
            now = time.perf_counter()
            if t_flag is None and (rc != 0 or int(flag[0]) == rep + 1):
                t_flag = now
            if t_copy is None and hip.hipEventQuery(d1) == 0:
                t_copy = now
            if t_end is None and hip.hipEventQuery(k1) == 0:
                t_end = now
            if now - t0 > 2.0:
                break
        hip.hipDeviceSynchronize()
        kms = elapsed(k0, k1)
        f = lambda t: None if t is None else round((t - t_issue) * 1e3, 4)  # noqa: E731
        rows.append({"kernel_ms": round(kms, 4), "flag_ms_after_issue": f(t_flag) if rc == 0 else f"rc {rc}",
                     "sdma_4B_ms_after_issue": f(t_copy), "grid_end_ms_after_issue": f(t_end)})
    emit({"probe": "B_flag_under_full_grid", "grid": "1400.hmm x 100k resident (" + e1400.variant_for(n) + ")",
          "issued_ms_after_grid_launch": 0.2, "reps": rows})
    e100.close()
    e1400.close()


if __name__ == "__main__":
    main()
