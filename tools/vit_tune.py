"""Time every compiled Viterbi-stage variant (vit_kernel.hip) that covers a profile on one batch, interleaved
rounds in one process, and check that they agree bitwise.  The batch: the MSV filter's survivors (P <= F1)
of bench.py's rank-0 batch of a config (--config), or --n random sequences.

    python tools/vit_tune.py --config cfg3 [--variants a,b] [--rounds 3] [--longest-first]
    python tools/vit_tune.py --profile 2405.hmm --n 2000 --lmin 1500 --lmax 2500
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OPS_PER_CELL = 14
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="")
    ap.add_argument("--profile", default="1400.hmm")
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--lmin", type=int, default=300)
    ap.add_argument("--lmax", type=int, default=500)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--F1", type=float, default=0.02)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="")
    ap.add_argument("--insert-mode", type=int, default=0)
    ap.add_argument("--in-place", action="store_true",
                    help="with --config: keep the WHOLE batch on the device and time each variant on the survivors "
                         "list msv_filter_select_device makes from the MSV launch's scores (bench.py's viterbi_stage "
                         "setting: scattered survivor residues, select indirection) instead of a compacted copy")
    ap.add_argument("--config-n", type=int, default=0, help="with --config: that config's first N sequences only")
    ap.add_argument("--sort-select", action="store_true",
                    help="with --in-place: re-list the device survivors exactly longest first (host sort, uploaded)")
    ap.add_argument("--longest-first", action="store_true",
                    help="survivors listed longest first (as msv_filter_select_device with the MSV order lists them)")
    a = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    native = _native.lib()
    native.msv_vit_debug_time_next_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    hip.hipEventDestroy.argtypes = [C.c_void_p]
    if a.config:
        prof, n, lmin, lmax, seed, scaling = CONFIGS[a.config]
        codes, offsets = random_batch(seed * 1000 if scaling == "weak" else seed, n, lmin, lmax)
        if a.config_n:
            offsets = offsets[:a.config_n + 1].copy()
            codes = codes[:int(offsets[-1])]
    else:
        prof = a.profile
        codes, offsets = random_batch(a.seed, a.n, a.lmin, a.lmax)
        if a.longest_first:  # the same residues re-cut with the lengths in descending order
            offsets[1:] = np.cumsum(np.sort(np.diff(offsets.astype(np.int64)))[::-1]).astype(np.uint64)
    h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
    sel_dev = None
    if a.config and a.in_place:  # bench.py's setting: the survivors selected on the device, in place
        dev = torch.device("cuda:0")
        m = msv.MSV_HMM(h)
        n_all = len(offsets) - 1
        r_all = torch.from_numpy(codes).to(dev)
        o_all = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s_all = torch.empty(n_all, dtype=torch.float32, device=dev)
        order = torch.empty(n_all, dtype=torch.int32, device=dev)
        sel = torch.empty(n_all, dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        st0 = torch.cuda.Stream(dev)
        m.reserve_length(int(np.diff(offsets.astype(np.int64)).max()))
        m.order_longest_first(o_all.data_ptr(), n_all, order.data_ptr(), st0.cuda_stream)
        m.score_batch_device(r_all.data_ptr(), r_all.numel(), o_all.data_ptr(), n_all, s_all.data_ptr(),
                             order.data_ptr(), st0.cuda_stream)
        native.msv_filter_select_device.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_float,
                                                    C.c_float, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _native.check(native.msv_filter_select_device(0, s_all.data_ptr(), o_all.data_ptr(), order.data_ptr(), n_all,
                                                      m.msv_mu, m.msv_lambda, a.F1, None, sel.data_ptr(), cnt.data_ptr(),
                                                      st0.cuda_stream))
        torch.cuda.synchronize()
        k = int(cnt.item())
        keep = np.sort(sel[:k].cpu().numpy().view(np.uint32).astype(np.int64))
        if a.sort_select:
            lens_all = np.diff(offsets.astype(np.int64))
            srt = keep[np.argsort(-lens_all[keep], kind="stable")].astype(np.uint32)
            sel[:k].copy_(torch.from_numpy(srt.view(np.int32)))
            torch.cuda.synchronize()
        sel_dev = (r_all, o_all, sel, cnt, n_all)
        cells_res = int(np.diff(offsets.astype(np.int64))[keep].sum())
    elif a.config:  # the survivors of the MSV filter
        m = msv.MSV_HMM(h)
        sc = m.score_batch(codes=codes, offsets=offsets)
        keep = np.nonzero(m.pvalues(sc, offsets) <= a.F1)[0]
        if a.longest_first:
            keep = keep[np.argsort(-np.diff(offsets.astype(np.int64))[keep], kind="stable")]
        parts = [codes[int(offsets[i]):int(offsets[i + 1])] for i in keep]
        offs = np.zeros(len(keep) + 1, np.uint64)
        np.cumsum([len(p) for p in parts], out=offs[1:])
        codes, offsets = np.concatenate(parts), offs
    n = len(offsets) - 1
    leng = h.model_length - 1
    cells = (cells_res if sel_dev is not None else int(offsets[-1])) * leng
    vit = msv.Viterbi_HMM(h, insert_mode=a.insert_mode)
    import re

    def states(v):  # team variants vit_w<W>_s<S>_*: W waves of 64 lanes x S states
        m = re.match(r"vit_(?:w(\d+)_)?s(\d+)_", v)
        return 64 * int(m.group(2)) * int(m.group(1) or 1)

    names = a.variants.split(",") if a.variants else [
        v for v in vit.variants() if (v.endswith("i") == bool(a.insert_mode)) and states(v) >= leng]
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    if sel_dev is not None:
        r, o, d_sel, d_cnt, n = sel_dev
        sel_ptr, cnt_ptr = d_sel.data_ptr(), d_cnt.data_ptr()
    else:
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        sel_ptr = cnt_ptr = None
    s = torch.full((n,), float("-inf"), dtype=torch.float32, device=dev)
    vit.reserve_length(int(np.diff(offsets.astype(np.int64)).max()))
    res = {nm: [] for nm in names}
    ref = None
    same = {}
    for rnd in range(a.rounds):
        for nm in names:
            vit.set_variant(nm)
            for _ in range(2):
                vit.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), sel_ptr, cnt_ptr,
                                       stream=st.cuda_stream)
            evs = []
            for _ in range(a.reps):
                e0, e1 = C.c_void_p(), C.c_void_p()
                hip.hipEventCreate(C.byref(e0))
                hip.hipEventCreate(C.byref(e1))
                native.msv_vit_debug_time_next_launch(vit._p, e0, e1)
                vit.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), sel_ptr, cnt_ptr,
                                       stream=st.cuda_stream)
                evs.append((e0, e1))
            vit.check(st.cuda_stream)
            torch.cuda.synchronize()
            for e0, e1 in evs:
                t = C.c_float()
                hip.hipEventElapsedTime(C.byref(t), e0, e1)
                res[nm].append(float(t.value))
                hip.hipEventDestroy(e0)
                hip.hipEventDestroy(e1)
            got = s.cpu().numpy().view(np.uint32).copy()
            if ref is None:
                ref = got
            same[nm] = bool(np.array_equal(got, ref))
    for nm in names:
        ms = float(np.median(res[nm]))
        info = None
        vit.set_variant(nm)
        info = vit.describe()
        print(json.dumps({"profile": prof, "config": a.config or None, "longest_first": a.longest_first,
                          "in_place": a.in_place, "sort_select": a.sort_select,
                          "sequences": n, "residues": int(offsets[-1]),
                          "variant": nm, "ms_med": round(ms, 4), "ms_min": round(min(res[nm]), 4),
                          "gcups": round(cells / (ms * 1e-3) / 1e9, 1),
                          "valu_frac": round(OPS_PER_CELL * cells / (ms * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4),
                          "blocks": info["blocks"], "waves_per_block": info["waves_per_block"],
                          "bitwise_same": same[nm]}), flush=True)


if __name__ == "__main__":
    main()
