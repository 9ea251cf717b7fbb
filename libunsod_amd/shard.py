"""Partitioning a packet batch across GPUs.

Packets are independent, so a batch splits into contiguous per-rank ranges and
every rank folds its own range with no collective: uniform configs by packet
count, mixed-length configs by bytes (prefix sum over lengths, cut at
k * sum / world).  The only cross-rank traffic is the optional host-side sum of
bad-checksum counters and the max-over-ranks of the timing.
"""
from __future__ import annotations

import numpy as np


def shard_uniform(n: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) packet range of ``rank`` when every packet costs the same."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    return n * rank // world, n * (rank + 1) // world


def shard_by_bytes(lengths, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) packet range of ``rank`` with contiguous ranges balanced by
    bytes: range k ends at the first packet whose prefix sum reaches
    (k+1) * total / world."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    lens = np.asarray(lengths, np.int64)
    n = lens.size
    if n == 0:
        return 0, 0
    csum = np.cumsum(lens)
    total = int(csum[-1])

    def cut(k: int) -> int:
        if k <= 0:
            return 0
        if k >= world:
            return n
        return int(np.searchsorted(csum, total * k / world, side="left")) + 1

    lo, hi = cut(rank), cut(rank + 1)
    return min(lo, n), min(max(hi, lo), n)


def all_shards(lengths, world: int) -> list[tuple[int, int]]:
    return [shard_by_bytes(lengths, world, r) for r in range(world)]


def job_totals(elapsed_s: float, nbytes: float, npkts: float, device=None) -> tuple[float, float, float]:
    """Across the process group (if any): (max elapsed, sum bytes, sum packets).

    The only collective the checksum path uses -- timing bookkeeping, not data.
    ``device`` is where the reduction tensors live (a CUDA device for nccl/RCCL,
    None = CPU for gloo)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(elapsed_s), float(nbytes), float(npkts)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([nbytes, npkts], dtype=torch.float64, device=device)
    dist.all_reduce(s)
    return float(t.item()), float(s[0].item()), float(s[1].item())
