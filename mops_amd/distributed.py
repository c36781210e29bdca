"""Multi-GPU particle sharding (one process per GPU, torch.distributed/RCCL).

The reference has no real multi-device path (its MPI loop runs the whole job
on every rank, CLI/main.cpp:86).  Here particles are independent, the mesh
and snapshots are replicated in every GPU's HBM, particles are split into
contiguous shards, and the only exchange is a gather of the record slabs
at record instants -- issued on a side stream so it
overlaps the next segment's kernel.

A rank's ``ParticleSet`` keeps its state and records PHYSICALLY in locality
(slot) order: slot s holds local particle ``ids[s]``.  Slabs are gathered in
that order together with each rank's ``ids`` (once per call, after the
locality sort), and ``unshard_slots`` maps them back to global particle order.
"""
from __future__ import annotations

import numpy as np


def _is_torch(a) -> bool:
    # (numpy >= 2 arrays also have a `.device` attribute, so test the type)
    return type(a).__module__.split(".")[0] == "torch"


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
    if _is_torch(gathered):
        import torch
        return torch.cat(parts, dim=-1)
    return np.concatenate(parts, axis=-1)


def unshard_slots(gathered, gathered_ids, n_total: int, world: int):
    """Slot-ordered shards -> [..., n_total] in global particle order.

    ``gathered`` [world, ..., n_pad]: rank r's slab in its slot order;
    ``gathered_ids`` [world, n_pad]: rank r's ``ParticleSet.ids`` (slot -> local
    particle index within the rank's shard ``shard_bounds(n_total, r, world)``).
    """
    is_torch = _is_torch(gathered)
    if is_torch:
        import torch
        out = torch.empty(tuple(gathered.shape[1:-1]) + (int(n_total),), dtype=gathered.dtype, device=gathered.device)
    else:
        out = np.empty(tuple(gathered.shape[1:-1]) + (int(n_total),), dtype=gathered.dtype)
    seen = 0
    for r in range(world):
        lo, hi = shard_bounds(n_total, r, world)
        ids = gathered_ids[r][: hi - lo]
        ids = ids.long() if is_torch else np.asarray(ids, dtype=np.int64)
        if hi > lo and (int(ids.min()) < 0 or int(ids.max()) >= hi - lo):
            raise ValueError(f"rank {r}: slot ids outside its shard")
        # a permutation of the shard: each local id exactly once (a duplicate would leave another
        # particle's column unwritten)
        counts = (torch.bincount(ids, minlength=hi - lo) if is_torch else np.bincount(ids, minlength=hi - lo))
        if hi > lo and not bool((counts == 1).all()):
            raise ValueError(f"rank {r}: slot ids are not a permutation of its shard")
        out[..., lo + ids] = gathered[r][..., : hi - lo]
        seen += hi - lo
    if seen != n_total:
        raise ValueError("shards do not cover n_total")
    return out
