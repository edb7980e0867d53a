"""Kernel time with the residue stream read straight from page-locked HOST memory (the device alias of a
pinned buffer, no H2D copy) against the same batch resident in HBM; scores must be bitwise equal.

    python tools/zero_copy_probe.py --config cfg3 [--variant NAME] [--time 10]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--variant", default="")
    ap.add_argument("--time", type=int, default=10)
    ap.add_argument("--offsets-host", action="store_true", help="offsets from pinned host memory too")
    a = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native  # noqa: F401  (binds torch's HIP runtime)
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    hip = C.CDLL("libamdhip64.so.7")
    hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]

    def dev_alias(t):
        p = C.c_void_p()
        assert hip.hipHostGetDevicePointer(C.byref(p), C.c_void_p(t.data_ptr()), 0) == 0
        return p.value

    prof, n, lmin, lmax, seed = CONFIGS[a.config][:5]
    e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
    if a.variant:
        e.set_variant(a.variant)
    codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    d_res = torch.from_numpy(codes).to(dev)
    h_res = torch.from_numpy(codes).pin_memory()
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    h_off = torch.from_numpy(offsets.view(np.int64)).pin_memory()
    s1 = torch.empty(n, dtype=torch.float32, device=dev)
    s2 = torch.empty(n, dtype=torch.float32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    e.reserve_length(lmax)
    e.order_longest_first(d_off.data_ptr(), n, order.data_ptr(), st.cuda_stream)
    res_alias = dev_alias(h_res)
    off_ptr = dev_alias(h_off) if a.offsets_host else d_off.data_ptr()

    def timed(res_ptr, offp, out, k):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for x, y in ev:
            x.record(st)
            e.score_batch_device(res_ptr, int(offsets[-1]), offp, n, out.data_ptr(), order.data_ptr(), st.cuda_stream)
            y.record(st)
        e.check(st.cuda_stream)
        return sorted(x.elapsed_time(y) for x, y in ev)

    for _ in range(3):  # warm (clock)
        timed(d_res.data_ptr(), d_off.data_ptr(), s1, 5)
        timed(res_alias, off_ptr, s2, 2)
    hbm = timed(d_res.data_ptr(), d_off.data_ptr(), s1, a.time)
    host = timed(res_alias, off_ptr, s2, a.time)
    same = bool(np.array_equal(s1.cpu().numpy().view(np.uint32), s2.cpu().numpy().view(np.uint32)))
    print(json.dumps({"config": a.config, "variant": e.describe()["variant"], "residues": int(offsets[-1]),
                      "offsets_from_host": a.offsets_host, "hbm_ms_median": hbm[len(hbm) // 2],
                      "host_zero_copy_ms_median": host[len(host) // 2], "bitwise_same": same}), flush=True)


if __name__ == "__main__":
    main()
