"""Does a HIP graph shorten bench.py's step (longest-first order + one MSV launch, resident in HBM)?
Times K steps launched on a stream against K replays of the same two launches captured once in a HIP
graph (torch.cuda.CUDAGraph over the library's launches on the capturing stream), and checks the scores.

    python tools/graph_probe.py --config cfg2 [--steps 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    from bench import CONFIGS

    prof, n, lmin, lmax, seed = CONFIGS[a.config][:5]
    e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
    codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
    dev = torch.device("cuda:0")
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(dev)
    e.reserve_length(lmax)
    e.bind_stream(st.cuda_stream)
    torch.cuda.synchronize()

    def step():
        e.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
        e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(), st.cuda_stream)

    def timed(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3

    ms_stream = timed(step)
    want = s.cpu().numpy().copy()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        step()  # the launch slots in use before capture are settled
        st.synchronize()
        s.fill_(float("nan"))
        with torch.cuda.graph(g, stream=st):
            step()
    torch.cuda.synchronize()
    ms_graph = timed(g.replay)
    e.check(st.cuda_stream)
    same = bool(np.array_equal(s.cpu().numpy().view(np.uint32), want.view(np.uint32)))
    ms_stream2 = timed(step)
    print(json.dumps({"config": a.config, "ms_per_step_stream": ms_stream, "ms_per_step_graph": ms_graph,
                      "ms_per_step_stream_again": ms_stream2, "graph_scores_bitwise_same": same}), flush=True)


if __name__ == "__main__":
    main()
