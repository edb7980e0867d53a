"""Timeline of msv_score_batch's host pipeline for rocprofv3 --kernel-trace --memory-copy-trace:
`--calls` warm calls of one config's batch from pinned memory, the last `--mark` of them after a
1 ms host sleep so they stand apart in the trace.

    rocprofv3 --kernel-trace --memory-copy-trace -d out -o run -- python3 tools/host_pipeline_trace.py
    python3 tools/pipeline_timeline.py out/run_kernel_trace.csv out/run_memory_copy_trace.csv

--per-sequence PROFILE instead times the reference's own call pattern: parallel_run_on_sequence once per
sequence of random_FASTA.fsa (3 x 3,500 residues, pageable, benchmark_MSV_1400.cpp:8-13).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--mark", type=int, default=3)
    ap.add_argument("--streamed", type=int, default=0,
                    help="after the one-call passes: a 1 ms gap, then this many msv_score_batch_async calls, three in flight")
    ap.add_argument("--per-sequence", default="")
    a = ap.parse_args()
    import torch
    import bench  # noqa: F401  (sets GPU_MAX_HW_QUEUES before HIP starts)
    import hmm_fasta_viterbi_amd as msv
    if a.per_sequence:
        e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", a.per_sequence)))
        fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "random_FASTA.fsa"))
        for k in range(a.calls):
            if k >= a.calls - a.mark:
                time.sleep(0.001)
            t = time.perf_counter()
            e.parallel_run_on_sequence(fa.sequences[k % len(fa.sequences)])
            print(f"call {k}: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
        return
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    prof, n, lmin, lmax, seed, _ = bench.CONFIGS[a.config]
    e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
    codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
    pinned = torch.from_numpy(codes).pin_memory().numpy()
    pout = torch.empty(n, dtype=torch.float32).pin_memory().numpy()
    for k in range(a.calls):
        if k >= a.calls - a.mark:
            time.sleep(0.001)
        t = time.perf_counter()
        e.score_batch(codes=pinned, offsets=offsets, out=pout)
        print(f"call {k}: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
    if a.streamed:
        outs = [torch.empty(n, dtype=torch.float32).pin_memory().numpy() for _ in range(3)]
        time.sleep(0.001)
        t = time.perf_counter()
        inflight = []
        for k in range(a.streamed):
            inflight.append(e.score_batch_async(pinned, offsets, outs[k % 3]))
            if len(inflight) == 3:
                e.wait(inflight.pop(0))
        for tk in inflight:
            e.wait(tk)
        dt = (time.perf_counter() - t) * 1e3
        print(f"streamed: {a.streamed} calls {dt:.3f} ms = {dt / a.streamed:.3f} ms per call", flush=True)


if __name__ == "__main__":
    main()
