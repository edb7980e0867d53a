"""Host->device copy rates on the GPU box, for the host-buffer scoring path (msv_score_batch).

    python tools/micro/h2d_bw.py [--mb 40] [--reps 10]

Prints one JSON line per case: pageable / pinned (torch pin_memory) sources, one copy or
pieces of `--piece-mb`, each the mean of `--reps` copies after one warm copy, timed with the
host clock around a stream synchronize.  Diagnostic only (not part of bench.py's value).
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch


def timed(fn, stream, reps):
    fn()
    stream.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    stream.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=40)
    ap.add_argument("--piece-mb", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    nbytes = a.mb << 20
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    host = np.random.default_rng(0).integers(0, 20, nbytes, dtype=np.uint8)
    pageable = torch.from_numpy(host)
    pinned = pageable.pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    piece = a.piece_mb << 20

    def whole(src):
        def f():
            with torch.cuda.stream(st):
                d.copy_(src, non_blocking=True)
        return f

    def pieces(src):
        def f():
            with torch.cuda.stream(st):
                for k in range(0, nbytes, piece):
                    d[k:k + piece].copy_(src[k:k + piece], non_blocking=True)
        return f

    for name, fn in (("pageable", whole(pageable)), ("pinned", whole(pinned)),
                     ("pageable_pieces", pieces(pageable)), ("pinned_pieces", pieces(pinned))):
        s = timed(fn, st, a.reps)
        print(json.dumps({"case": name, "MB": a.mb, "piece_MB": a.piece_mb if "pieces" in name else None,
                          "ms": round(s * 1e3, 4), "GBps": round(nbytes / s / 1e9, 2)}), flush=True)
    # device -> host (scores) for scale
    small = torch.empty(100_000, dtype=torch.float32, device=dev)
    hs = torch.empty(100_000, dtype=torch.float32).pin_memory()

    def d2h():
        with torch.cuda.stream(st):
            hs.copy_(small, non_blocking=True)
    s = timed(d2h, st, a.reps)
    print(json.dumps({"case": "d2h_pinned_400KB", "ms": round(s * 1e3, 4)}), flush=True)
    assert torch.equal(d.cpu(), pageable)


if __name__ == "__main__":
    main()
