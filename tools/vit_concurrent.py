"""Feasibility probe: the Viterbi launch's drain tail filled by a second, concurrent launch.  The survivors
list (cfg3, host-compacted, longest first) is split: the head [0, n - K) runs as one launch of the pick
(`--head`, one wave per sequence), the tail [n - K, n) as a launch of a small-workgroup team variant
(`--tail`) on a second stream, forked after and joined before the head's stream; its workgroups can only
start as the head launch's waves leave.  Time from the fork to the join (torch events) against the whole
list as one launch; scores bitwise equal.

    python tools/vit_concurrent.py --config cfg3 --head vit_w1_s22_ea --tail vit_w2_s11_g1 --ks 0,512,1024
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--head", default="vit_w1_s22_ea")
    ap.add_argument("--tail", default="vit_w2_s11_g1")
    ap.add_argument("--ks", default="0,256,512,1024,1536,2048,3072")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--F1", type=float, default=0.02)
    a = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    prof, n, lmin, lmax, seed, scaling = CONFIGS[a.config]
    codes, offsets = random_batch(seed * 1000 if scaling == "weak" else seed, n, lmin, lmax)
    h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
    m = msv.MSV_HMM(h)
    sc = m.score_batch(codes=codes, offsets=offsets)
    keep = np.nonzero(m.pvalues(sc, offsets) <= a.F1)[0]
    keep = keep[np.argsort(-np.diff(offsets.astype(np.int64))[keep], kind="stable")]
    m.close()
    dev = torch.device("cuda:0")
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    d_res = torch.from_numpy(codes).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    ns = len(keep)
    d_sel = torch.from_numpy(keep.astype(np.int32)).to(dev)
    vh, vt = msv.Viterbi_HMM(h), msv.Viterbi_HMM(h)
    vh.set_variant(a.head)
    vt.set_variant(a.tail)
    for v in (vh, vt):
        v.reserve_length(lmax)
    ref = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
    out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
    cnt = {}

    def count(k):
        if k not in cnt:
            cnt[k] = torch.tensor([k], dtype=torch.int32, device=dev)
        return cnt[k]

    def run(k, dst):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(sa)
        if ns - k > 0:
            vh.score_batch_device(d_res.data_ptr(), d_res.numel(), d_off.data_ptr(), n, dst.data_ptr(),
                                  d_sel.data_ptr(), count(ns - k).data_ptr(), sa.cuda_stream)
        if k > 0:
            sb.wait_event(e0)
            vt.score_batch_device(d_res.data_ptr(), d_res.numel(), d_off.data_ptr(), n, dst.data_ptr(),
                                  d_sel[ns - k:].data_ptr(), count(k).data_ptr(), sb.cuda_stream)
            e1.record(sb)
            sa.wait_event(e1)
        e2.record(sa)
        return e0, e2

    torch.cuda.synchronize()
    run(0, ref)
    torch.cuda.synchronize()
    vh.check(sa.cuda_stream)
    ks = [int(x) for x in a.ks.split(",")]
    times = {k: [] for k in ks}
    for rep in range(a.reps):
        for k in ks:
            e0, e2 = run(k, out)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e2))
            if rep == 0:
                same = bool(torch.equal(out[d_sel.long()], ref[d_sel.long()]))
                times[k].append(same)
    for k in ks:
        same = times[k].pop(1)
        t = np.array(times[k][1:] if len(times[k]) > 2 else times[k], np.float64)
        print(json.dumps({"config": a.config, "survivors": ns, "head": a.head, "tail": a.tail, "tail_k": k,
                          "ms_med": round(float(np.median(t)), 4), "ms_min": round(float(t.min()), 4),
                          "bitwise_same": same}), flush=True)


if __name__ == "__main__":
    main()
