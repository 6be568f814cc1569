"""Multi-GPU sharding of the MSM: point-partition across ranks, all-gather of the
per-rank partial sums (one 64-B WrappedPoint each), combine by elliptic-curve addition.

RCCL (torch.distributed "nccl") has no EC-point reduction operator, so the collective is an
all-gather of the partials followed by a device-side sum (halo_point_sum).  There is no data-path
collective: every rank reads only its own resident SRS block and scalars.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of points owned by `rank` (SRS block r, scalars r)."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def allgather_points(partial: np.ndarray, dist, device=None) -> np.ndarray:
    """All-gather one WrappedPoint (8 x u64) per rank -> (world, 8) uint64 array."""
    import torch

    world = dist.get_world_size()
    t = torch.from_numpy(np.ascontiguousarray(partial, dtype=np.uint64).view(np.int64).copy())
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.stack([p.cpu().numpy().view(np.uint64) for p in parts])


def sharded_msm(partial_msm: Callable[[int, int], np.ndarray], point_sum: Callable[[np.ndarray], np.ndarray],
                n_total: int, dist, device=None) -> np.ndarray:
    """MSM over n_total points split across ranks: each rank computes partial_msm(lo, hi) over its
    block, partials are all-gathered and summed with point_sum (identical result on every rank)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_range(n_total, rank, world)
    part = partial_msm(lo, hi)
    if world == 1:
        return part
    return point_sum(allgather_points(part, dist, device))
