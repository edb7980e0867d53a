"""Per-wave / per-sequence timeline of one Viterbi team-kernel launch (diagnostic: msv_vit_debug_set_stamps).
Where a launch's time goes beyond its steady state: table staging, the first sequences, and the drain tail
(how long SIMDs hold 3 / 2 / 1 / 0 of their waves).

    python tools/vit_timeline.py --config cfg3                      # the MSV survivors, longest first
    python tools/vit_timeline.py --n 3072 --lmin 400 --lmax 400     # random 1400.hmm batch, longest first
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(x):
    x = np.asarray(x, np.float64)
    return [round(float(np.percentile(x, p)), 1) for p in (0, 1, 10, 50, 90, 99, 100)] if len(x) else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="")
    ap.add_argument("--profile", default="1400.hmm")
    ap.add_argument("--n", type=int, default=3072)
    ap.add_argument("--lmin", type=int, default=300)
    ap.add_argument("--lmax", type=int, default=500)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--variant", default="")
    ap.add_argument("--F1", type=float, default=0.02)
    a = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    lib = _native.lib()
    lib.msv_vit_debug_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
    if a.config:
        prof, n, lmin, lmax, seed, scaling = CONFIGS[a.config]
        codes, offsets = random_batch(seed * 1000 if scaling == "weak" else seed, n, lmin, lmax)
        h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
        m = msv.MSV_HMM(h)
        sc = m.score_batch(codes=codes, offsets=offsets)
        keep = np.nonzero(m.pvalues(sc, offsets) <= a.F1)[0]
        keep = keep[np.argsort(-np.diff(offsets.astype(np.int64))[keep], kind="stable")]
        parts = [codes[int(offsets[i]):int(offsets[i + 1])] for i in keep]
        offsets = np.zeros(len(keep) + 1, np.uint64)
        np.cumsum([len(p) for p in parts], out=offsets[1:])
        codes = np.concatenate(parts)
        m.close()
    else:
        prof = a.profile
        codes, offsets = random_batch(a.seed, a.n, a.lmin, a.lmax)
        offsets[1:] = np.cumsum(np.sort(np.diff(offsets.astype(np.int64)))[::-1]).astype(np.uint64)
        h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
    n = len(offsets) - 1
    vit = msv.Viterbi_HMM(h)
    if a.variant:
        vit.set_variant(a.variant)
    info = vit.describe()
    nw = info["blocks"] * info["waves_per_block"]
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    stamps = torch.zeros((n + nw) * 4, dtype=torch.int64, device=dev)
    vit.reserve_length(int(np.diff(offsets.astype(np.int64)).max()))
    torch.cuda.synchronize()
    for _ in range(2):
        vit.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), None, None, st.cuda_stream)
    lib.msv_vit_debug_set_stamps(vit._p, stamps.data_ptr())
    vit.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), None, None, st.cuda_stream)
    vit.check(st.cuda_stream)
    lib.msv_vit_debug_set_stamps(vit._p, None)
    torch.cuda.synchronize()
    x = stamps.cpu().numpy().view(np.uint64).reshape(n + nw, 4).astype(np.int64)
    seq, wav = x[:n], x[n:]
    if (wav[:, 2] == 0).any() or (seq[:, 1] == 0).any():
        sys.exit("timeline incomplete (not a team-kernel variant?)")
    t0 = wav[:, 0].min()
    us = lambda t: (t - t0) / 100.0  # s_memrealtime: 100 MHz
    entry, staged, exit_ = us(wav[:, 0]), us(wav[:, 1]), us(wav[:, 2])
    T = float(exit_.max())
    xcc = wav[:, 3]
    s0, s1 = us(seq[:, 0]), us(seq[:, 1])
    hw = seq[:, 2] >> 32
    gw = seq[:, 2] & 0xFFFFFFFF
    L = seq[:, 3].astype(np.float64)
    # SIMD key: XCC, SE, SH, CU, SIMD (gfx9 HW_ID fields) of the wave that ran the sequence
    simd_of_wave = {}
    for j in range(n):
        h_ = int(hw[j])
        simd_of_wave[int(gw[j])] = (int(xcc[gw[j]]), (h_ >> 13) & 7, (h_ >> 12) & 1, (h_ >> 8) & 15, (h_ >> 4) & 3)
    keys = sorted(set(simd_of_wave.values()))
    kidx = {k: i for i, k in enumerate(keys)}
    # active waves per SIMD over time (a wave is active from its first sequence's start to its last one's end)
    first = np.full(nw, np.inf)
    last = np.zeros(nw)
    nseq = np.zeros(nw, int)
    np.minimum.at(first, gw, s0)
    np.maximum.at(last, gw, s1)
    np.add.at(nseq, gw, 1)
    grid = np.linspace(0, T, 2001)
    act = np.zeros((len(keys), len(grid)), int)
    for w in np.nonzero(nseq)[0]:
        k = kidx[simd_of_wave[int(w)]]
        act[k] += (grid >= first[w]) & (grid < last[w])
    share = {c: round(float((act == c).mean()), 4) for c in range(int(act.max()) + 1)}
    # per-sequence ns per row, by its ordinal on its wave and by the mean active waves on its SIMD
    order = np.lexsort((s0, gw))
    ordinal = np.zeros(n, int)
    prev = -1
    c = 0
    for j in order:
        c = c + 1 if gw[j] == prev else 0
        prev = gw[j]
        ordinal[j] = c
    nspr = (s1 - s0) * 1000.0 / np.maximum(L, 1)
    mean_act = np.zeros(n)
    for j in range(n):
        k = kidx[simd_of_wave[int(gw[j])]]
        sel = (grid >= s0[j]) & (grid < s1[j])
        mean_act[j] = act[k, sel].mean() if sel.any() else np.nan
    drained = float(s0.max())  # the last sequence's start: the list is empty after it
    res = {
        "profile": prof, "config": a.config or None, "variant": info["variant"], "sequences": n, "waves": nw,
        "residues": int(offsets[-1]), "launch_us": round(T, 1),
        "entry_us": pct(entry), "tables_staged_us": pct(staged), "staging_us": pct(staged - entry),
        "first_sequence_start_us": pct(first[nseq > 0]),
        "list_drained_at_us": round(drained, 1), "tail_after_drain_us": round(T - drained, 1),
        "wave_exit_us": pct(exit_),
        "simd_time_share_by_active_waves": share,
        "ns_per_row_by_ordinal": {int(k): pct(nspr[ordinal == k]) for k in range(int(ordinal.max()) + 1)},
        "ns_per_row_by_active_waves": {str(b): pct(nspr[np.round(mean_act) == b]) for b in (1, 2, 3, 4)
                                       if (np.round(mean_act) == b).any()},
        "sequences_per_wave": pct(nseq),
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
