"""cfg2's row, segment by segment: shader cycles per row of the 16-lane, 8-state plan's short-row
loop, split into [0] residue block + prologue (Bt, the j-1 neighbour's DPP move) + the 8 cells, [1] the epilogue
(lane E tree, J, N, B, cursor), [2] the wave-level rare-event test and its branch -- from the plan's CLOCK twin in
a timing-only build that stamps s_memtime at those boundaries (tools/ab_patches/r06_msv_row_segments.patch, built
with EXTRA_DEVFLAGS=-DMSV_SEGMENTS; the stamps' waits perturb the row, so the tool reports the twin's own row time
beside the production kernel's).

Batches: the one-wave-per-SIMD floor batch (4,096 x 500 residues: 1,024 waves of 4 sequences) and cfg2's own
(bench.py's rank-0 batch, 10,000 x U[300, 500]).

    MSV_LIB_PATH=abx/r6seg/libmsv_hip.so python tools/cfg2_segments.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WORDS = 10


def main():
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", "100.hmm")))
    native = _native.lib()
    native.msv_debug_time_next_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    native.msv_debug_set_clock_stamps.argtypes = [C.c_void_p, C.c_void_p]
    native.msv_debug_grid_waves.argtypes = [C.c_void_p]
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    eng.bind_stream(st.cuda_stream)
    nwaves = int(native.msv_debug_grid_waves(eng._p))

    def ev():
        e = C.c_void_p()
        assert hip.hipEventCreate(C.byref(e)) == 0
        return e.value

    def run(codes, offsets, label, launches=12):
        n = len(offsets) - 1
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s = torch.empty(n, dtype=torch.float32, device=dev)
        order = torch.empty(n, dtype=torch.int32, device=dev)
        buf = torch.zeros(nwaves * WORDS, dtype=torch.int64, device=dev)
        out = {"batch": label, "variant": eng.variant_for(n)}
        for mode in ("production", "twin"):
            times, segs = [], []
            for k in range(launches + 5):
                eng.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
                pair = (ev(), ev())
                native.msv_debug_time_next_launch(eng._p, pair[0], pair[1])
                if mode == "twin":
                    buf.zero_()
                    native.msv_debug_set_clock_stamps(eng._p, buf.data_ptr())
                eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(),
                                       st.cuda_stream)
                native.msv_debug_set_clock_stamps(eng._p, None)
                st.synchronize()
                if k >= 5:
                    t = C.c_float()
                    assert hip.hipEventElapsedTime(C.byref(t), pair[0], pair[1]) == 0
                    times.append(float(t.value))
                    if mode == "twin":
                        a = buf.cpu().numpy().view(np.uint64).reshape(nwaves, WORDS)
                        a = a[a[:, 9] > 0]
                        rows = a[:, 9].astype(np.float64)
                        clock = (a[:, 5] - a[:, 4]).astype(np.float64).sum() / (a[:, 1] - a[:, 0]).astype(np.float64).sum() * 0.1
                        segs.append([float((a[:, 6 + q].astype(np.float64)).sum() / rows.sum()) for q in range(3)]
                                    + [clock, float(rows.sum() / len(a)), len(a)])
            eng.check(st.cuda_stream)
            out[mode + "_ms"] = round(float(np.median(times)), 4)
            if mode == "twin":
                m = np.median(np.array(segs), axis=0)
                out["clock_GHz"] = round(float(m[3]), 3)
                out["cycles_per_row"] = {"cells": round(float(m[0]), 1), "epilogue": round(float(m[1]), 1),
                                         "event_test": round(float(m[2]), 1),
                                         "total": round(float(m[0] + m[1] + m[2]), 1)}
                out["rows_per_wave"] = round(float(m[4]), 1)
                out["waves_stamped"] = int(m[5])
        print(json.dumps(out), flush=True)

    run(*random_batch(77, 4096, 500, 500), "floor 4096 x 500 (one wave per SIMD)")
    run(*random_batch(1000, 10000, 300, 500), "cfg2 10000 x U[300,500]")


if __name__ == "__main__":
    main()
