"""Run the Viterbi stage alone on a BASELINE config's MSV survivors, as the pipeline lists them (for
rocprofv3 --kernel-trace / --pmc passes of vit_kernel): the MSV launch (longest-first order), the
survivors selected on the device in that order (P <= F1), then `--launches` Viterbi launches.

    python tools/run_vit.py --config cfg3 --launches 3 [--variant vit_s22_t5a]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--variant", default="")
    ap.add_argument("--F1", type=float, default=0.02)
    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    prof, n, lmin, lmax, seed, scaling = CONFIGS[args.config]
    h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
    m = msv.MSV_HMM(h)
    vit = msv.Viterbi_HMM(h)
    if args.variant:
        vit.set_variant(args.variant)
    codes, offsets = random_batch(seed * 1000 if scaling == "weak" else seed, n, lmin, lmax)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    sh = st.cuda_stream
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    sel = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    vs = torch.empty(n, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    m.reserve_length(lmax)
    vit.reserve_length(lmax)
    m.order_longest_first(o.data_ptr(), n, order.data_ptr(), sh)
    m.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(), sh)
    _native.check(_native.lib().msv_filter_select_device(0, s.data_ptr(), o.data_ptr(), order.data_ptr(), n,
                                                         m.msv_mu, m.msv_lambda, args.F1, None, sel.data_ptr(),
                                                         cnt.data_ptr(), sh))
    for _ in range(args.launches):
        vit.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, vs.data_ptr(), sel.data_ptr(),
                               cnt.data_ptr(), sh)
    vit.check(sh)
    torch.cuda.synchronize()
    print(f"{vit.describe()['variant']}: {int(cnt.item())} survivors, {args.launches} launches", flush=True)


if __name__ == "__main__":
    main()
