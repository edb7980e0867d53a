"""Multi-GPU sharding of an MSV batch: one process per GPU (torch.distributed; backend "nccl" is
RCCL over xGMI on MI355X, "gloo" on CPU for tests).

Sequences are independent, so the batch is cut into contiguous shards with equal
residue counts (a prefix-sum split, which keeps the output order), each rank scores its shard
with ONE fused kernel launch, and the per-sequence float scores are gathered once at the end
(4 B per sequence; the only collective, it carries outputs, never DP state).  The reference has
no multi-device path at all ("Parallelism strategies: none").
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def shard_bounds(offsets: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """[first, last) sequence range of `rank` with ~equal residues per rank (contiguous)."""
    offsets = np.asarray(offsets, np.uint64)
    n = len(offsets) - 1
    if world <= 1:
        return 0, n
    total = int(offsets[-1] - offsets[0])
    cuts = [0]
    for r in range(1, world):
        target = offsets[0] + (total * r) // world
        cuts.append(int(np.searchsorted(offsets[1:], target, side="left")))
    cuts.append(n)
    for r in range(1, world + 1):  # monotone
        cuts[r] = max(cuts[r], cuts[r - 1])
    return cuts[rank], cuts[rank + 1]


def shard(codes: np.ndarray, offsets: np.ndarray, world: int, rank: int):
    """The rank's (codes, rebased offsets, first, last)."""
    first, last = shard_bounds(offsets, world, rank)
    lo, hi = int(offsets[first]), int(offsets[last])
    offs = (np.asarray(offsets[first:last + 1], np.uint64) - np.uint64(lo)).astype(np.uint64)
    return codes[lo:hi], offs, first, last


def score_sharded(scorer: Callable[[np.ndarray, np.ndarray], np.ndarray], codes: np.ndarray, offsets: np.ndarray,
                  device=None) -> np.ndarray:
    """Score a batch across all ranks of the default process group and return every score on
    every rank.  `scorer(codes, offsets) -> float32 scores` runs on this rank's shard (e.g.
    MSV_HMM.score_batch bound to this rank's GPU).  `device` is where the collective's tensors
    live ("cuda:<local>" for RCCL, None/"cpu" for gloo)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    n = len(offsets) - 1
    c, o, first, last = shard(codes, offsets, world, rank)
    local = np.asarray(scorer(c, o), np.float32) if last > first else np.zeros(0, np.float32)
    if world == 1:
        return local
    bounds = [shard_bounds(offsets, world, r) for r in range(world)]
    width = max(b - a for a, b in bounds)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    buf = torch.full((width,), float("nan"), dtype=torch.float32, device=dev)
    if local.size:
        buf[: local.size] = torch.from_numpy(local).to(dev)
    out = torch.empty(world * width, dtype=torch.float32, device=dev)
    dist.all_gather_into_tensor(out, buf)
    out = out.cpu().numpy().reshape(world, width)
    res = np.empty(n, np.float32)
    for r, (a, b) in enumerate(bounds):
        res[a:b] = out[r, : b - a]
    return res
