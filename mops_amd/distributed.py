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


def all_gather_flat(dist, out, inp, backend: str, group=None):
    """One all-gather of a rank's flat slab into ``out`` ([world * inp.numel()]).  nccl (RCCL over
    xGMI) runs on the caller's current stream; gloo (CPU tests, one-GPU rehearsals) stages device
    tensors through host memory."""
    if backend == "nccl" or not out.is_cuda:
        dist.all_gather_into_tensor(out, inp, group=group)
    else:
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)


def gather_flat(dist, out, inp, backend: str, world: int, rank: int, dst: int = 0, group=None):
    """One gather of every rank's flat slab into ``out`` ([world * inp.numel()]) on rank ``dst`` only
    (SURVEY.md §8e's "Gather to rank 0").  nccl (RCCL) runs it as point-to-point sends over each
    sender's direct xGMI link to the root, on the caller's current stream; gloo stages device tensors
    through host memory.  ``out`` is ignored on the other ranks (None allowed)."""
    import torch
    if backend == "nccl" or not inp.is_cuda:
        gl = list(out.view(world, -1).unbind(0)) if rank == dst else None
        dist.gather(inp, gather_list=gl, dst=dst, group=group)
    else:
        gl = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(world)] if rank == dst else None
        dist.gather(inp.cpu(), gather_list=gl, dst=dst, group=group)
        if rank == dst:
            out.view(world, -1).copy_(torch.stack(gl))


# xGMI: 7 point-to-point links per MI355X, ~153 GB/s each (one process per GPU on one node)
XGMI_LINK_GBS = 153.0


def gather_seconds(sent_bytes: float, world: int, link_gbs: float = XGMI_LINK_GBS) -> dict:
    """Modeled seconds of one checkpoint's exchange when every rank contributes ``sent_bytes`` (DESIGN.md
    section 7's table).  xGMI is point-to-point, so the models differ in how many links carry the bytes:

    - all_gather_ring: a single ring, every rank receives (world-1) slabs through one link;
    - all_gather_direct: fully connected, each rank receives each peer's slab over that peer's own link, all
      links at once (the lower bound for any all-gather);
    - root_direct: Gather to rank 0, every sender over its own link to the root, in parallel;
    - root_serial: the root's receives one after another (the upper bound for the gather).

    Every rank's HBM takes (world-1) slabs in an all-gather, only rank 0's in a gather."""
    w = int(world)
    if w <= 1:
        return {"link_gbs": link_gbs, "all_gather_ring": 0.0, "all_gather_direct": 0.0, "root_direct": 0.0,
                "root_serial": 0.0}
    one = float(sent_bytes) / (link_gbs * 1e9)
    return {"link_gbs": link_gbs, "all_gather_ring": (w - 1) * one, "all_gather_direct": one, "root_direct": one,
            "root_serial": (w - 1) * one}


class RecordGather:
    """The north star's trajectory collection: at every checkpoint -- the end of a
    StreamLine call or of a chained pathline pair -- each rank's record slab is all-gathered, so
    every rank holds the records of every particle.

    A rank's ``ParticleSet`` keeps its records in slot (locality) order, so each checkpoint also
    gathers, per slot, the run's seed (x, y, z) and the slot's particle id: with them
    ``lines()`` rebuilds every line in global particle order (``unshard_slots`` +
    ``mops_traj_finalize``), bit-identical to a single-rank run.

    Overlap: ``collect`` swaps the particle set onto a second record slab (``ParticleSet.
    swap_records``), so the next call writes one slab while the comm stream gathers the other; the
    compute stream waits for a slab's gather only when that slab comes back a call later.  The
    seeds and ids are copied into one of two aux buffers on the compute stream first (the next
    call's reseed and re-sort rewrite them in place).

    Bounded memory: a checkpoint's gathered records (world x K x 48 B per particle) can exceed what HBM
    holds beside the fields (config 5 at 8 ranks: 149 GB per pair); with ``max_bytes`` the slab is
    all-gathered in chunks of records through a ring of that size, in order on the comm stream, and
    ``on_chunk(gathered, k0, k1)`` (enqueued on the comm stream before the next chunk overwrites the ring)
    is where an output writer takes each chunk.

    ``mode``: "all" (the default: all_gather, every rank holds every record) or "root" (Gather to rank 0:
    only rank 0 receives, allocates the ring, calls ``on_chunk`` and can rebuild lines; every sender uses
    its own xGMI link, DESIGN.md section 7 models both).

    Torch device tensors (RCCL, or gloo staged through the host) and CPU tensors (gloo tests)."""

    # PathlineChain.run refuses defer_lines with an on_pair that reads the pair's record slab:
    # collect() does, and a bound method exposes its function's attributes (set below the class)
    reads_records = True

    def __init__(self, dist, ps, world: int, backend: str = "nccl", comm_stream=None, group=None,
                 max_bytes: int | None = None, on_chunk=None, mode: str = "all"):
        import torch
        if mode not in ("all", "root"):
            raise ValueError("RecordGather mode: 'all' or 'root'")
        self.dist, self.world, self.backend, self.group = dist, int(world), backend, group
        self.mode = mode
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.receives = mode == "all" or self.rank == 0
        self.torch = torch
        self.shape = tuple(ps.records.shape)            # [K_max][6][stride]
        self.stride = self.shape[2]
        dev = ps.records.device
        self.cuda = ps.records.is_cuda
        self.comm = comm_stream if (comm_stream is not None or not self.cuda) else torch.cuda.Stream(dev)
        self.spare = torch.empty(self.shape, dtype=torch.float64, device=dev)
        self.aux = [torch.zeros((4, self.stride), dtype=torch.float64, device=dev) for _ in range(2)]
        per_rec = self.world * 6 * self.stride * 8
        self.chunk = self.shape[0] if not max_bytes else max(1, min(self.shape[0], int(max_bytes) // per_rec))
        if self.world > 1:  # every rank must issue the same collectives: the smallest chunk of all ranks
            t = torch.tensor([self.chunk], dtype=torch.int64,
                             device=dev if (backend == "nccl" and self.cuda) else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
            self.chunk = int(t.item())
        self.on_chunk = on_chunk
        wr = self.world if self.receives else 0  # (root mode: the senders hold no ring)
        self.gathered = torch.empty((wr, self.chunk, 6, self.stride), dtype=torch.float64, device=dev)
        self.gathered_aux = torch.empty((wr, 4, self.stride), dtype=torch.float64, device=dev)
        self.gather_events = []  # (start, end) comm-stream events of every checkpoint's exchange (CUDA)
        self._read = {}      # id(slab / aux) -> comm-stream event after the gather that read it
        self._i = 0
        self.K = 0            # records of the last gathered checkpoint
        self.n = ps.n
        self.done = None      # comm-stream event: the last checkpoint is in `gathered`
        self.checkpoints = 0
        self.bytes_per_rank = 0  # bytes each rank sent so far

    def _wait(self, stream, key):
        ev = self._read.pop(key, None)
        if ev is not None and stream is not None:
            stream.wait_event(ev)

    def collect(self, ps, compute=None):
        """Gather ``ps``'s current records (its first ``ps.K`` slots), seeds and slot ids; ``compute``:
        the stream the particle set's work is ordered on (None: CPU)."""
        torch = self.torch
        if tuple(ps.records.shape) != self.shape:
            raise ValueError("particle set record slab changed shape")
        aux = self.aux[self._i]
        self._i ^= 1
        ctx = torch.cuda.stream(compute) if (self.cuda and compute is not None) else _null()
        with ctx:
            self._wait(compute, id(aux))  # its previous gather has read it
            n = ps.n
            aux[0:3, :n].copy_(ps.seeds.t())
            aux[3, :n].copy_(ps.ids.to(torch.float64))
            if n < self.stride:
                aux[3, n:].fill_(-1.0)
            slab = ps.records
            self._wait(compute, id(self.spare))  # the slab about to be written again has been gathered
            self.spare = ps.swap_records(self.spare)
            ready = None
            if self.cuda:
                ready = torch.cuda.Event()
                ready.record(compute if compute is not None else torch.cuda.current_stream(slab.device))
        K = int(ps.K)
        cctx = torch.cuda.stream(self.comm) if self.cuda else _null()
        if self.cuda:
            self.comm.wait_event(ready)
        with cctx:
            if self.cuda:
                t0 = torch.cuda.Event(enable_timing=True)
                t0.record(self.comm)
            self._exchange(self.gathered_aux.view(-1), aux.view(-1))
            row = 6 * self.stride
            for k0 in range(0, K, self.chunk):
                k1 = min(K, k0 + self.chunk)
                m = (k1 - k0) * row
                self._exchange(self.gathered.view(-1)[: self.world * m] if self.receives else None,
                               slab.view(-1)[k0 * row: k1 * row])
                if self.on_chunk is not None and self.receives:
                    self.on_chunk(self.gathered.view(-1)[: self.world * m].view(self.world, k1 - k0, 6, self.stride),
                                  k0, k1)
            if self.cuda:
                t1 = torch.cuda.Event(enable_timing=True)
                t1.record(self.comm)
                self.gather_events.append((t0, t1))
                ev = torch.cuda.Event()
                ev.record(self.comm)
                self._read[id(slab)] = ev
                self._read[id(aux)] = ev
                self.done = ev
        self.K = K
        self.checkpoints += 1
        self.bytes_per_rank += (K * 6 + 4) * self.stride * 8
        return self.done

    def _exchange(self, out, inp):
        if self.mode == "all":
            all_gather_flat(self.dist, out, inp, self.backend, self.group)
            return
        try:
            gather_flat(self.dist, out, inp, self.backend, self.world, self.rank, 0, self.group)
        except (RuntimeError, NotImplementedError, ValueError) as e:
            if self.checkpoints > 0 or inp.numel() != 4 * self.stride:  # (only the first exchange: the aux slab)
                raise
            # a backend without Gather (it refuses before any byte moves, on every rank alike): fall back to the
            # all-gather before the first exchange, with every rank's ring allocated
            import sys
            print(f"[RecordGather] gather to rank 0 unavailable ({e}); all-gather instead", file=sys.stderr)
            torch = self.torch
            self.mode, self.receives = "all", True
            dev = self.spare.device
            self.gathered = torch.empty((self.world, self.chunk, 6, self.stride), dtype=torch.float64, device=dev)
            self.gathered_aux = torch.empty((self.world, 4, self.stride), dtype=torch.float64, device=dev)
            all_gather_flat(self.dist, self.gathered_aux.view(-1), inp, self.backend, self.group)

    def gather_ms(self) -> list:
        """Comm-stream milliseconds of every checkpoint's exchange so far (CUDA; call after synchronize)."""
        return [a.elapsed_time(b) for (a, b) in self.gather_events]

    def plan(self, compute_s_per_checkpoint: float | None = None) -> dict:
        """The per-rank memory plan of the collection (bench.py prints it for N > 1): bytes gathered per
        checkpoint (every rank's slab at the longest record count), the ring that receives them (the whole
        gathered slab, or chunks of records when max_bytes bounds it), the spare slab and aux buffers, and
        the HBM left beside the fields once they are allocated."""
        per_rec = self.world * 6 * self.stride * 8
        out = {"world": self.world, "records_per_checkpoint_max": self.shape[0],
               "gathered_bytes_per_checkpoint": per_rec * self.shape[0],
               "sent_bytes_per_checkpoint": (self.shape[0] * 6 + 4) * self.stride * 8,
               "ring_bytes": self.gathered.numel() * 8 + self.gathered_aux.numel() * 8,
               "ring_records": self.chunk, "chunked": self.chunk < self.shape[0],
               "spare_slab_bytes": self.spare.numel() * 8, "aux_bytes": sum(a.numel() for a in self.aux) * 8,
               "mode": self.mode,
               "received_bytes_per_checkpoint": ((self.world - 1) * (self.shape[0] * 6 + 4) * self.stride * 8
                                                 if self.receives else 0)}
        sent = (self.shape[0] * 6 + 4) * self.stride * 8
        model = gather_seconds(sent, self.world)
        out["modeled_seconds_per_checkpoint"] = model
        if compute_s_per_checkpoint:
            mine = model["all_gather_ring"] if self.mode == "all" else model["root_serial"]
            out["compute_seconds_per_checkpoint"] = compute_s_per_checkpoint
            out["modeled_gather_over_compute"] = {k: v / compute_s_per_checkpoint for k, v in model.items()
                                                  if k != "link_gbs"}
            out["modeled_worst_case_over_compute"] = mine / compute_s_per_checkpoint
        if self.gather_events:
            ms = self.gather_ms()
            out["measured_gather_ms"] = {"mean": sum(ms) / len(ms), "max": max(ms), "checkpoints": len(ms)}
        if self.cuda:
            free, total = self.torch.cuda.mem_get_info(self.spare.device)
            out.update(hbm_free_bytes=int(free), hbm_total_bytes=int(total))
        return out

    def synchronize(self):
        if self.cuda and self.comm is not None:
            self.comm.synchronize()

    def unsharded(self, n_total: int):
        """(records [K][6][n_total], seeds [n_total][3]) of the last checkpoint in global particle
        order (call after ``synchronize``; needs the whole slab in one chunk)."""
        K, w = self.K, self.world
        if not self.receives:
            raise ValueError("root mode: only rank 0 holds the gathered records")
        if K > self.chunk:
            raise ValueError("the last checkpoint was gathered in chunks (max_bytes): take them in on_chunk")
        g = self.gathered.view(-1)[: w * K * 6 * self.stride].view(w, K * 6, self.stride)
        ids = self.gathered_aux[:, 3, :].to(self.torch.int64)
        rec = unshard_slots(g, ids, n_total, w).view(K, 6, n_total)
        seeds = unshard_slots(self.gathered_aux[:, 0:3, :], ids, n_total, w).t().contiguous()
        return rec.contiguous(), seeds

    def lines(self, n_total: int, pathline: bool, stream=None):
        """Every particle's finalized line from the last checkpoint (device tensors; mops_traj_finalize
        over the unsharded records, identity line order): what a single-rank run's finalize returns."""
        import ctypes as C
        from . import _lib as L
        torch = self.torch
        rec, seeds = self.unsharded(n_total)
        K, P = self.K, self.K + 1
        dev = rec.device
        pts = torch.empty((n_total, P, 3), dtype=torch.float64, device=dev)
        vel = torch.empty_like(pts)
        tmp = torch.empty((n_total, P), dtype=torch.float64, device=dev)
        sal = torch.empty_like(tmp)
        last = torch.empty((n_total, 3), dtype=torch.float64, device=dev)
        st = 0 if stream is None else int(stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
        L.check(L.load().mops_traj_finalize(n_total, K, C.c_void_p(seeds.data_ptr()), C.c_void_p(rec.data_ptr()),
                                            n_total, 1 if pathline else 0, None, C.c_void_p(pts.data_ptr()),
                                            C.c_void_p(vel.data_ptr()), C.c_void_p(tmp.data_ptr()),
                                            C.c_void_p(sal.data_ptr()), C.c_void_p(last.data_ptr()), C.c_void_p(st)),
                "mops_traj_finalize")
        return dict(points=pts, velocity=vel, temperature=tmp, salinity=sal, lastPoint=last)


RecordGather.collect.reads_records = True  # (on_pair = rg.collect: a bound method reads its function's attributes)


def _null():
    import contextlib
    return contextlib.nullcontext()
