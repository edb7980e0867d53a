"""Per-wave timeline of one MSV launch (diagnostic build path: msv_debug_set_stamps).
Prints how long waves live relative to the launch (the tail), rows per wave, per-XCD spread.

    python tools/wave_timeline.py --config cfg3 [--variant NAME] [--no-order]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

STAMP_WORDS = 4  # msv_kernel_body.inc: realtime start/end, hwid|rows, xcc|block (production kernels)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--variant", default="")
    ap.add_argument("--no-order", action="store_true")


    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    L = _native.lib()
    L.msv_debug_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
    L.msv_debug_grid_waves.argtypes = [C.c_void_p]
    prof, n, lmin, lmax, seed = CONFIGS[args.config][:5]
    n = args.n or n
    eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
    if args.variant:
        eng.set_variant(args.variant)


    codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    nw = L.msv_debug_grid_waves(eng._p)
    stamps = torch.zeros(nw * STAMP_WORDS, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    if not args.no_order:
        eng.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
    op = None if args.no_order else order.data_ptr()
    eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), op, st.cuda_stream)  # warm
    L.msv_debug_set_stamps(eng._p, stamps.data_ptr())
    eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), op, st.cuda_stream)
    eng.check(st.cuda_stream)
    L.msv_debug_set_stamps(eng._p, None)
    a = stamps.cpu().numpy().reshape(nw, STAMP_WORDS)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    start = (a[:, 0] - t0) / 100.0  # us
    end = (a[:, 1] - t0) / 100.0
    T = end.max()
    rows = (a[:, 2] & 0xFFFFFFFF).astype(np.float64)
    hwid = (a[:, 2] >> 32).astype(np.int64)
    cu_key = (a[:, 3] >> 32).astype(np.int64) * 4096 + ((hwid >> 8) & 0xF) + 16 * ((hwid >> 12) & 0x1) + \
        32 * ((hwid >> 13) & 0x7)
    simd = (hwid >> 4) & 0x3
    _, waves_per_cu = np.unique(cu_key, return_counts=True)
    xcc = (a[:, 3] >> 32).astype(int)
    life = (end - start) / T
    q = lambda x: [round(float(np.percentile(x, p)), 1) for p in (0, 1, 10, 50, 90, 99, 100)]
    blk = (a[:, 3] & 0xFFFFFFFF).astype(int)
    W = eng.describe()["waves_per_block"]
    wid = np.zeros(len(a), int)
    # stamps are stored at index blockIdx*W + wave, recover wave-in-block from the row index
    idx = np.nonzero(stamps.cpu().numpy().reshape(nw, STAMP_WORDS)[:, 1] > 0)[0]
    wid = idx % W
    res_extra = {
        "distinct_cus": int(len(waves_per_cu)),
        "waves_per_cu_pct": q(waves_per_cu),
        "simd_of_wave_in_block": [int(np.bincount(simd[wid == w], minlength=4).argmax()) for w in range(W)],
        "rows_by_wave_in_block_median": [int(np.median(rows[wid == w])) for w in range(W)],
        "end_by_wave_in_block_median": [round(float(np.median(end[wid == w])), 0) for w in range(W)],
    }
    res = {
        "variant": eng.describe()["variant"], "order": not args.no_order,  "waves": int(len(a)),
        "launch_us": round(float(T), 1),
        "start_us_pct": q(start), "end_us_pct": q(end),
        "mean_wave_lifetime_frac": round(float(life.mean()), 4),
        "rows_per_wave_pct": q(rows),
        "ns_per_row_pct": q((end - start) * 1000.0 / np.maximum(rows, 1)),
        "waves_per_simd_pct": q(np.unique(cu_key * 4 + simd, return_counts=True)[1]),
        "end_us_by_xcc_median": {int(x): round(float(np.median(end[xcc == x])), 1) for x in sorted(set(xcc))},
        "end_us_by_xcc_max": {int(x): round(float(end[xcc == x].max()), 1) for x in sorted(set(xcc))},
    }
    res.update(res_extra)
    # the waves holding the batch's longest sequences (rows within 2% of the most): when they start, how fast
    # their rows ran (the floor is their rows at the one-wave-per-SIMD row time) and how many waves shared
    # their SIMD -- the decomposition of a latency-bound launch (cfg2) against its floor
    lw = rows >= 0.98 * rows.max()
    simd_key = cu_key * 4 + simd
    _, inv, cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
    res["longest_waves"] = {
        "count": int(lw.sum()), "rows": q(rows[lw]), "start_us_pct": q(start[lw]), "end_us_pct": q(end[lw]),
        "ns_per_row_pct": q((end[lw] - start[lw]) * 1000.0 / np.maximum(rows[lw], 1)),
        "waves_on_their_simd_pct": q(cnt[inv][lw]),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
