"""Multi-GPU particle sharding (one process per GPU, torch.distributed/RCCL).

The reference has no real multi-device path (its MPI loop runs the whole job
on every rank, CLI/main.cpp:86).  Here particles are independent, the mesh
and snapshots are replicated in every GPU's HBM, particles are split into
contiguous shards, and the only exchange is a gather of the record slabs
at record instants -- issued on a side stream so it
overlaps the next segment's kernel.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of particle indices owned by `rank`."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def max_shard(n_total: int, world: int) -> int:
    return -(-int(n_total) // int(world))


def record_slab_gather(slab, world: int, group=None, async_op: bool = False):
    """All-gather one record slab [6, n_pad] (same n_pad on every rank).

    Returns (gathered [world, 6, n_pad], work handle or None).  With the
    nccl (RCCL) backend this runs over xGMI on the caller's current stream.
    """
    import torch
    import torch.distributed as dist
    out = torch.empty((world,) + tuple(slab.shape), dtype=slab.dtype, device=slab.device)
    if world == 1:
        out[0].copy_(slab)
        return out, None
    work = dist.all_gather_into_tensor(out.view(-1), slab.contiguous().view(-1), group=group, async_op=async_op)
    return out, work


def unshard(gathered, n_total: int, world: int):
    """[world, ..., n_pad] gathered shards -> [..., n_total] in global particle order."""
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(n_total, r, world)
        parts.append(gathered[r][..., : hi - lo])
    if hasattr(gathered, "device"):
        import torch
        return torch.cat(parts, dim=-1)
    return np.concatenate(parts, axis=-1)
