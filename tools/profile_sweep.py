"""Kernel rate of every bundled profile on one resident batch (the cfg3 shape by default): which variant
each table size takes and how close it runs to the measured instruction ceiling.

    python tools/profile_sweep.py [--config cfg3] [--n N] [--time 10]

One JSON line per profile: the variant of the plan the batch size takes, kernel ms (median of
`--time` launches timed with HIP events on the launch stream, after 5 warm-up launches, longest-first
order), M residues/s, T cells/s (cells =
residues x LENG, as bench.py) and the fraction of the issue ceiling bench.py reports against
(21.469 T cells/s, profiles/r01_micro_row_sched.jsonl).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ISSUE_CEILING_TCELLS = 21.469


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--time", type=int, default=10)
    a = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    _, n, lmin, lmax, seed = CONFIGS[a.config][:5]
    n = a.n or n
    codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
    residues = int(offsets[-1])
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    pdir = os.path.join(ROOT, "data", "profile_HMMs")
    names = sorted(os.listdir(pdir), key=lambda f: int(f.split(".")[0]))
    for name in names:
        eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(pdir, name)))
        eng.reserve_length(lmax)
        eng.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
        for _ in range(5):
            eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(),
                                   st.cuda_stream)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.time)]
        for e0, e1 in ev:
            e0.record(st)
            eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(),
                                   st.cuda_stream)
            e1.record(st)
        eng.check(st.cuda_stream)
        ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)[a.time // 2]
        leng = eng.model_length - 1
        info = eng.describe()
        tcells = residues * leng / (ms * 1e-3) / 1e12
        info["variant"] = eng.variant_for(n)  # the plan this batch size takes
        print(json.dumps({"config": a.config, "profile": name, "LENG": leng, "n": n, "residues": residues,
                          "variant": info["variant"], "kernel_ms": round(ms, 4),
                          "M_residues_s": round(residues / (ms * 1e-3) / 1e6, 1), "tcells_s": round(tcells, 3),
                          "issue_ceiling_frac": round(tcells / ISSUE_CEILING_TCELLS, 4)}), flush=True)
        del eng


if __name__ == "__main__":
    main()
