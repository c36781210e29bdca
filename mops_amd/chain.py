"""Snapshot-pair chaining for long pathlines, device resident.

Host-side mirror of the reference's pair loop -- ``MOPSPathline.run``
(tutorial/pyMOPSAPI.py:1396-1531) and tutorial/pathLine.cpp:244-309 --
with the MI355X-specific change that nothing leaves HBM between pairs:

* snapshot i+2's derived field is built on a side stream while pair i runs,
  and a field is freed as soon as no pair needs it (at most 3 resident);
* the continuation seeds (each pair's ``lastPoint``), the per-particle
  depths and the concatenated lines stay device tensors.

Per-pair semantics are the reference's:
* pair p runs a PathLine with front = snapshot p, back = snapshot p+1 and
  ``simulationDuration`` = that pair's snapshot gap, |t(p+1) - t(p)| from the
  snapshots' timestamps (``_time_gap_seconds``, :1285-1295, :1444;
  tutorial/pathLine.cpp:287-305) -- calendar-month pairs (28-31 days,
  ``_month_pairs_forward/_backward``, :1236-1279) give every pair its own step
  and record count;
* seeds: pair 0 uses the given seeds, later pairs the previous pair's
  ``lastPoint`` if ``follow_last`` else the original seeds again (:1446-1459);
* depth: constant mode re-applies ``cfg.depth`` every pair (``cfg.depth =
  self._depth``, :1470); per-particle mode carries
  ``clip(EARTH_RADIUS_M - |lastPoint|, 0)`` as float32 (:1462-1467, 1486-1491);
* lines: pair 0's lines whole, later pairs without their first sample
  (:1500-1516); ``lastPoint`` = the last pair's.
"""
from __future__ import annotations

from datetime import datetime

import numpy as np

from . import _lib as L
from .engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig

EARTH_RADIUS_M = 6_371_000.0  # pyMOPSAPI.py:46
REORDER_SECONDS = 3 * 86400  # default launch length of long pairs (simulated time), see PathlineChain.run
XTIME_FORMAT = "%Y-%m-%d_%H:%M:%S"  # MPAS xtime (pyMOPSAPI.py:1285; Utils.hpp:118)


def month_pairs_forward(sy: int, sm: int, ey: int, em: int) -> list:
    """(start, end) month pairs 'YYYY-MM-01' from (sy, sm) up to (ey, em), forward in time --
    MOPSPathline._month_pairs_forward (tutorial/pyMOPSAPI.py:1236-1257; the C++ tutorial's
    MOPS_IO::make_forward_month_pairs, YamlGen.hpp:360-379, yields the same list)."""
    out = []
    y, m = int(sy), int(sm)
    while (y, m) <= (int(ey), int(em)):
        ny, nm = (y + 1, 1) if m == 12 else (y, m + 1)
        if (ny, nm) > (int(ey), int(em)):
            break
        out.append((f"{y:04d}-{m:02d}-01", f"{ny:04d}-{nm:02d}-01"))
        y, m = ny, nm
    return out


def month_pairs_backward(sy: int, sm: int, ey: int, em: int) -> list:
    """(start, end) month pairs from (sy, sm) back to (ey, em) -- MOPSPathline._month_pairs_backward
    (tutorial/pyMOPSAPI.py:1259-1279)."""
    out = []
    y, m = int(sy), int(sm)
    while (y, m) >= (int(ey), int(em)):
        py_, pm = (y - 1, 12) if m == 1 else (y, m - 1)
        if (py_, pm) < (int(ey), int(em)):
            break
        out.append((f"{y:04d}-{m:02d}-01", f"{py_:04d}-{pm:02d}-01"))
        y, m = py_, pm
    return out


def time_gap_seconds(t1: str, t2: str, fmt: str = XTIME_FORMAT) -> int:
    """t1 - t2 in seconds for MPAS timestamps, each cut at its first NUL and stripped
    (MOPSPathline._time_gap_seconds, tutorial/pyMOPSAPI.py:1285-1295; C++ getTimeGapinSecond,
    src/Utils/Utils.hpp:113-132)."""
    a = datetime.strptime(t1.split("\x00", 1)[0].strip(), fmt)
    b = datetime.strptime(t2.split("\x00", 1)[0].strip(), fmt)
    return int((a - b).total_seconds())


def pair_gaps(timestamps) -> list:
    """Each consecutive snapshot pair's simulationDuration, |t(p+1) - t(p)| (pyMOPSAPI.py:1444)."""
    ts = list(timestamps)
    return [abs(time_gap_seconds(ts[p + 1], ts[p])) for p in range(len(ts) - 1)]


def month_timestamps(pairs) -> list:
    """The snapshot timestamps of a month-pair list: each pair's start, then the last pair's end
    (the xtime of a monthly-mean file dated 'YYYY-MM-01', at 00:00:00)."""
    if not pairs:
        return []
    return [a + "_00:00:00" for a, _ in pairs] + [pairs[-1][1] + "_00:00:00"]


class PathlineChain:
    def __init__(self, mesh: DeviceMesh, make_field, n_snapshots: int, gap_seconds=None, device=None,
                 own_fields: bool = True, prefetch: bool = True, overlap_stream=None, timestamps=None):
        """``make_field(i, stream) -> DeviceField`` builds snapshot i's field on ``stream``.
        Pair p's simulationDuration: ``gap_seconds`` (one int for every pair, or a sequence with
        one gap per pair), or from the snapshots' ``timestamps`` (MPAS xtime strings, one per
        snapshot) as the reference computes it (``pair_gaps``).
        With ``own_fields`` False the fields are the caller's (e.g. all resident
        before a timed region) and are neither freed nor rebuilt here.
        ``prefetch`` builds snapshot p+2 on a side stream while pair p runs (3
        fields resident); without it, p+2 is built after pair p has freed
        snapshot p (2 resident: an oRRS18to6-class field at L=80 is ~75 GB).
        Without prefetch, a ``make_field`` with ``refill(field, i, stream)``
        (and optionally ``prepare(i)``, e.g. synth_device.DeviceFieldRecycler)
        re-derives snapshot p's buffers in place as p+2 instead -- no
        allocation and no host synchronisation between pairs.
        ``overlap_stream`` (with such a recycling ``make_field`` holding three
        field buffers): snapshot p+2 is generated and derived into the buffer
        pair p-1 released, on that stream while pair p computes -- give it CUs
        of its own (``cu_split_streams``): the trajectory waves fill every CU
        they may use, so a stream sharing them only runs once they drain."""
        if n_snapshots < 2:
            raise ValueError("a pathline chain needs at least two snapshots")
        self.mesh = mesh
        self.make_field = make_field
        self.n_snapshots = int(n_snapshots)
        if timestamps is not None:
            if len(timestamps) != self.n_snapshots:
                raise ValueError("one timestamp per snapshot")
            gaps = pair_gaps(timestamps)
        elif gap_seconds is None:
            raise ValueError("give gap_seconds or timestamps")
        elif np.isscalar(gap_seconds):
            gaps = [int(gap_seconds)] * (self.n_snapshots - 1)
        else:
            gaps = [int(g) for g in gap_seconds]
        if len(gaps) != self.n_snapshots - 1:
            raise ValueError("one gap per snapshot pair")
        self.gaps = gaps
        self.gap = gaps[0]
        self.device = device
        self.own_fields = own_fields
        self.prefetch = prefetch
        self.overlap_stream = overlap_stream

    def run(self, seeds, depth: float, particle_depths=None, method: int = L.MOPS_EULER, delta_t: int = 60,
            record_t: int = 360, direction: int = L.MOPS_FORWARD, follow_last: bool = True, keep_lines: bool = True,
            compute_stream=None, on_pair=None, timing=None, segment_steps: int = -1, reorder: bool = True,
            record_stride: int | None = None, defer_lines: bool = False, compact: bool | None = None,
            compact_chunks: int = 6, on_lines=None, lines_chunk: int | None = None):
        """Run all pairs; returns device tensors {points, velocity, temperature,
        salinity, lastPoint, death_step (of the last pair)} when ``keep_lines``,
        else only lastPoint/death_step.  ``on_pair(p, last, ps)`` is called after pair p
        is enqueued, with the pair's ParticleSet (its slot-ordered record slab, seeds and ids:
        the multi-GPU record gather, distributed.RecordGather); ``timing`` (a list) receives an
        (start, end) HIP event pair around every trajectory launch.
        ``attempted`` in the result counts particle-steps whose velocity
        evaluation ran, summed over pairs (device scalar).  ``segment_steps``: integration
        steps per kernel launch (0 = one launch per pair: every launch re-reads the particle
        state and re-loads each particle's cell stencil; -1 = one launch per REORDER_SECONDS
        of simulated time).  ``reorder``: restore the particles' locality order between
        launches (long pairs: particles drift across many cells and a wave's lanes stop
        sharing stencils -- config 5's 30-day pairs run 9% faster re-sorted every 3 days).
        ``record_stride``: columns of the record slab (default n; a multi-GPU shard pads it to the
        largest shard so every rank's slab gathers with one all-gather).  ``defer_lines``: each pair's lines
        are assembled on a side stream beside the next pair, from a second record slab and side copies of
        the seeds and slot ids; the next pair's seeds come from mops_traj_last_points (the same doubles as
        the assembly's lastPoint).  ``on_pair`` then sees the set after the slab swap, so an ``on_pair``
        that reads ``ps.records`` (an attribute ``reads_records`` = True, e.g. a distributed.RecordGather
        collector) is refused with it.
        ``compact``: dead-particle compaction (ParticleSet.compact) between ``compact_chunks`` launches per
        pair -- live particles re-sorted to the front in locality order, the launch spread over them only;
        None = on for RK4, whose stages must stay in the step's start cell (quirk Q1: a particle dies at its
        first cell crossing, ~0.8 per particle-day at config 3).  Result-invariant.
        ``on_lines(p, lines, ids)``: a writer hook instead of concatenating the lines in HBM (the reference
        caller's lines_acc, pyMOPSAPI.py:1497-1518): each pair's lines are assembled in chunks of
        ``lines_chunk`` particle slots (default all) and handed over as device tensors {points, velocity,
        temperature, salinity} -- pairs after the first without their first sample, as the reference
        appends them -- with ``ids`` (int32 device tensor: the particle of each row).  The chunk buffers
        are reused: the hook consumes or copies them, on the current (compute) stream, before returning.
        The next pair's seeds come from mops_traj_last_points.  Not with ``keep_lines`` or ``defer_lines``."""
        import torch
        if on_lines is not None and (keep_lines or defer_lines):
            raise ValueError("on_lines hands each pair's lines to the hook: not with keep_lines or defer_lines")
        if defer_lines and on_pair is not None and getattr(on_pair, "reads_records", False):
            raise ValueError("defer_lines swaps the record slab before on_pair: an on_pair that reads ps.records "
                             "(reads_records) would see the next pair's slab")
        do_compact = (int(method) == L.MOPS_RK4) if compact is None else bool(compact)
        dev = self.device or torch.device("cuda", torch.cuda.current_device())
        cs = compute_stream or torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(device=dev)
        cfgs = [TrajectoryConfig(deltaT=int(delta_t), simulationDuration=int(g), recordT=int(record_t),
                                 depth=float(np.float32(depth)), direction=int(direction), method=int(method))
                for g in self.gaps]
        for c in cfgs:
            if c.n_steps <= 0 or c.n_records <= 0:
                raise ValueError("invalid trajectory settings for a pair (deltaT/recordT vs the snapshot gap "
                                 f"{c.simulationDuration} s)")
        # the particle set's record slab holds the longest pair's records; each pair runs with its own
        # simulationDuration (steps, records, the alpha ramp)
        cfg = max(cfgs, key=lambda c: c.n_records)
        # everything below is ordered on `cs` (the host never waits between pairs, so a
        # tensor touched on another stream could be read before `cs` has written it)
        with torch.cuda.stream(cs):
            if isinstance(seeds, torch.Tensor):  # (device-resident seeds: no upload; the set copies them)
                seeds0 = seeds.to(device=dev, dtype=torch.float64).reshape(-1, 3).contiguous()
            else:
                seeds0 = torch.as_tensor(np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 3), device=dev)
            n = int(seeds0.shape[0])
            per_particle = particle_depths is not None and len(particle_depths) == n
            pdep = (torch.as_tensor(np.asarray(particle_depths, dtype=np.float32), device=dev) if per_particle
                    else None)

        recycle = self.own_fields and not self.prefetch and hasattr(self.make_field, "refill")
        overlap = recycle and self.overlap_stream is not None
        if overlap and self.n_snapshots > 2 and not hasattr(self.make_field, "pool"):
            raise ValueError("overlap_stream needs a recycling make_field with a buffer pool "
                             "(synth_device.DeviceFieldRecycler)")
        fields = {}
        with torch.cuda.stream(cs):
            fields[0] = self.make_field(0, cs.cuda_stream)
            fields[1] = self.make_field(1, cs.cuda_stream)
            if overlap and self.n_snapshots > 2 and len(self.make_field.pool) < 1:
                raise ValueError("overlap_stream needs a third field buffer in make_field.pool (seed the "
                                 "recycler with three fields and release them before the run)")
            ps = ParticleSet(self.mesh, seeds0, cfg.depth, cfg, device=dev, record_stride=record_stride)
        period = ps.record_period(pathline=True)
        pts_acc, vel_acc, tmp_acc, sal_acc = [], [], [], []
        last = None
        attempted = torch.zeros((), dtype=torch.int64, device=dev)
        ov = self.overlap_stream
        ready, pair_done = {}, {}
        asm = torch.cuda.Stream(device=dev) if defer_lines else None
        dl = dict(slab=None, seeds=None, ids=None, assembled=None)  # the deferred assembly's buffers
        for p in range(self.n_snapshots - 1):
            if overlap and p + 2 < self.n_snapshots:
                # snapshot p+2 into the buffer pair p-1 released (pair 0: the third pooled buffer)
                buf = self.make_field.pool.pop() if p == 0 else fields.pop(p - 1)
                if p > 0:
                    ov.wait_event(pair_done.pop(p - 1))
                with torch.cuda.stream(ov):
                    fields[p + 2] = self.make_field.refill(buf, p + 2, ov)
                    ready[p + 2] = torch.cuda.Event()
                    ready[p + 2].record(ov)
            if p + 1 in ready:
                cs.wait_event(ready.pop(p + 1))  # pair p's back snapshot was derived on the overlap stream
            with torch.cuda.stream(cs):
                if p == 0 or not follow_last:
                    s = seeds0
                else:
                    s = last
                if per_particle:
                    if p > 0:
                        # the reference updates the depths from every pair's last points, whether or not the
                        # next seeds follow them (pyMOPSAPI.py:1490-1495; with follow_last the pre-run update
                        # at :1465-1469 recomputes the same values from seeds = lastPoint).
                        # np.linalg.norm(axis=1) order: sqrt((x*x + y*y) + z*z)
                        r = torch.sqrt((last[:, 0] * last[:, 0] + last[:, 1] * last[:, 1]) + last[:, 2] * last[:, 2])
                        pdep = torch.clamp(EARTH_RADIUS_M - r, min=0.0).to(torch.float32)
                    d = pdep
                else:
                    d = cfg.depth
                cfg = cfgs[p]
                ps.set_config(cfg)
                # a continuation pair: each particle's current cell is an exact-locate hint
                ps.reseed(s, d, stream=cs.cuda_stream, hint_cells=(p > 0 and follow_last))
                front, back = fields[p], fields[p + 1]
                if (not overlap and recycle and p + 2 < self.n_snapshots
                        and hasattr(self.make_field, "prepare")):
                    # raw snapshot p+2 generated on a side stream beside pair p's first launch (started
                    # earlier, its blocks would fill the GPU ahead of the reseed's small kernels)
                    started = torch.cuda.Event()
                    started.record(cs)
                    self.make_field.prepare(p + 2, after=started)
                if segment_steps < 0:
                    seg = max(1, REORDER_SECONDS // int(delta_t))
                else:
                    seg = cfg.n_steps if segment_steps == 0 else int(segment_steps)  # records by absolute step
                bounds = set(range(0, cfg.n_steps, seg))
                if do_compact:
                    ch = max(1, int(compact_chunks))
                    bounds |= {cfg.n_steps * k // ch for k in range(ch)}
                bounds = sorted(bounds) + [cfg.n_steps]
                live = None
                for s0, s1 in zip(bounds[:-1], bounds[1:]):
                    if s1 <= s0:
                        continue
                    if do_compact and s0 > 0:
                        # live particles first (locality order), the dead after them; the launch covers the
                        # live ones only.  Records written so far: slot 0's step-0 part .. the last completed
                        # record (as ParticleSet.advance_pipelined)
                        nrec = min(cfg.n_records, s0 // period + 1) if period else 1
                        live = ps.compact(0, ps.n, cs, records_written=nrec)
                    elif reorder and s0 > 0:
                        # every record slot moves with its particle: a particle that died earlier in the
                        # pair already holds the reference's zeros in its later slots
                        ps.reorder(stream=cs.cuda_stream)
                    if timing is not None:  # (the launch alone: what rocprofv3 averages)
                        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(cs)
                    ps.advance(front, back, s0, s1, stream=cs.cuda_stream, live_count=live)
                    if timing is not None:
                        e1.record(cs)
                        timing.append((e0, e1))
                if defer_lines:
                    last = ps.last_points(stream=cs.cuda_stream)
                    done_ev = torch.cuda.Event()
                    done_ev.record(cs)
                    asm.wait_event(done_ev)
                    if dl["slab"] is None:
                        dl.update(slab=torch.empty_like(ps.records), seeds=torch.empty_like(ps.seeds),
                                  ids=torch.empty_like(ps.ids))
                    if dl["assembled"] is not None:
                        cs.wait_event(dl["assembled"])  # the spare slab's last reader is done before it is rewritten
                    slab = ps.swap_records(dl["slab"])
                    with torch.cuda.stream(asm):
                        dl["seeds"].copy_(ps.seeds)
                        dl["ids"].copy_(ps.ids)
                    copied = torch.cuda.Event()
                    copied.record(asm)
                    cs.wait_event(copied)  # the next reseed rewrites seeds and ids in place
                    with torch.cuda.stream(asm):
                        out = ps.finalize_from(dl["seeds"], dl["ids"], slab, pathline=True, stream=asm.cuda_stream)
                    if keep_lines:
                        # allocated on `asm`, read on `cs` by the concatenation below (after cs.wait_stream(asm)):
                        # the allocator must not hand the blocks back to `asm` while `cs` may still read them
                        for t in out.values():
                            t.record_stream(cs)
                    dl["assembled"] = torch.cuda.Event()
                    dl["assembled"].record(asm)
                    dl["slab"] = slab
                elif on_lines is not None:
                    last = ps.last_points(stream=cs.cuda_stream)
                    self._hand_lines(ps, p, on_lines, lines_chunk, cs)
                else:
                    out = ps.finalize(pathline=True, stream=cs.cuda_stream)
                    last = out["lastPoint"].clone()
                dth = ps.death.to(torch.int64)
                attempted += torch.where(dth < 0, torch.full_like(dth, cfg.n_steps), dth + 1).sum()
                if keep_lines:
                    sl = slice(None) if p == 0 else slice(1, None)
                    pts_acc.append(out["points"][:, sl]); vel_acc.append(out["velocity"][:, sl])
                    tmp_acc.append(out["temperature"][:, sl]); sal_acc.append(out["salinity"][:, sl])
            if on_pair is not None:
                on_pair(p, last, ps)
            if overlap:
                pair_done[p] = torch.cuda.Event()
                pair_done[p].record(cs)  # snapshot p's buffer is free once pair p has run
                continue
            if recycle:  # re-derive snapshot p's buffers as snapshot p+2, stream-ordered after pair p
                if p + 2 < self.n_snapshots:
                    fields[p + 2] = self.make_field.refill(fields.pop(p), p + 2, cs)
                continue
            # overlap: build the field pair p+1 will need while pair p computes
            if p + 2 < self.n_snapshots and (self.prefetch or not self.own_fields):
                if self.own_fields:
                    with torch.cuda.stream(side):
                        fields[p + 2] = self.make_field(p + 2, side.cuda_stream)
                    cs.wait_stream(side)
                else:
                    fields[p + 2] = self.make_field(p + 2, cs.cuda_stream)
            done = fields.pop(p)
            if self.own_fields:
                cs.synchronize()  # pair p finished with `done` before it is freed
                done.close()
                if p + 2 < self.n_snapshots and not self.prefetch:
                    with torch.cuda.stream(cs):
                        fields[p + 2] = self.make_field(p + 2, cs.cuda_stream)
        if self.own_fields:
            cs.synchronize()
            if ov is not None:
                ov.synchronize()
            for f in fields.values():
                if hasattr(self.make_field, "release"):
                    self.make_field.release(f)  # kept for the next run (e.g. DeviceFieldRecycler)
                else:
                    f.close()
        if asm is not None:
            cs.wait_stream(asm)  # the last pair's lines
        with torch.cuda.stream(cs):
            res = dict(lastPoint=last, death_step=ps.original(ps.death), attempted=attempted)
            if keep_lines:
                res.update(points=torch.cat(pts_acc, 1), velocity=torch.cat(vel_acc, 1),
                           temperature=torch.cat(tmp_acc, 1), salinity=torch.cat(sal_acc, 1))
        if cs != torch.cuda.current_stream(dev):
            torch.cuda.current_stream(dev).wait_stream(cs)  # results are read on the caller's stream
        return res


    @staticmethod
    def _hand_lines(ps, p: int, on_lines, lines_chunk, cs):
        """Pair p's lines to the writer hook, assembled in chunks of particle slots (run(on_lines=...))."""
        import torch
        n = ps.n
        ch = n if not lines_chunk else max(1, min(int(lines_chunk), n))
        P = ps.K + 1
        dev = ps.seeds.device
        bufs = getattr(ps, "_line_bufs", None)
        if bufs is None or bufs["points"].shape[0] < ch or bufs["points"].shape[1] != P:
            with torch.cuda.stream(cs):
                bufs = dict(points=torch.empty((ch, P, 3), dtype=torch.float64, device=dev),
                            velocity=torch.empty((ch, P, 3), dtype=torch.float64, device=dev),
                            temperature=torch.empty((ch, P), dtype=torch.float64, device=dev),
                            salinity=torch.empty((ch, P), dtype=torch.float64, device=dev))
            ps._line_bufs = bufs
        sl = slice(None) if p == 0 else slice(1, None)  # later pairs without their first sample (:1512-1516)
        with torch.cuda.stream(cs):
            for lo in range(0, n, ch):
                hi = min(n, lo + ch)
                out = {k: v[:hi - lo] for k, v in bufs.items()}
                ps.finalize_range(lo, hi, out, pathline=True, stream=cs.cuda_stream)
                on_lines(p, {k: v[:, sl] for k, v in out.items()}, ps.ids[lo:hi])


class HostLineSink:
    """A ``PathlineChain.run(on_lines=...)`` writer hook that delivers every pair's lines to host memory, as
    the reference returns them to its caller (``MOPSApp::runPathLine`` -> ``vector<TrajectoryLine>``,
    src/Core/MOPSApp.cpp:254-337; pyMOPS -> ``list[dict]``, tools/pyMOPS/bindings.cpp:383-455;
    ``MOPSPathline.run`` accumulates them per pair, tutorial/pyMOPSAPI.py:1497-1518).

    Overlap: each chunk of lines is first copied on the compute stream into one of two device staging slabs
    (a device-to-device copy at HBM speed), then a copy stream moves that slab into pinned host buffers while
    the next pair computes.  Pair p uses slot p % 2 (device staging and host buffers alike); before pair p
    writes a slot, the compute stream waits for the host copy of pair p - 2 out of it.  So a caller reads
    pair p's host lines (``host(p)``) after ``synchronize()`` or after pair p + 1 was handed, and has until
    pair p + 2's lines arrive to consume them (``keep_all=True`` instead keeps every pair's host copy).

    ``ids[p]`` (host int32): the particle of each row (the chain hands lines in slot order)."""

    def __init__(self, n: int, k_max: int, device, keep_all: bool = False):
        import torch
        self.torch = torch
        self.n, self.P = int(n), int(k_max) + 1
        self.dev = torch.device(device)
        self.copy = torch.cuda.Stream(self.dev)
        self.keep_all = keep_all
        self.stage = [self._bufs(self.dev) for _ in range(2)]
        self.hostbufs = [] if keep_all else [self._bufs("cpu") for _ in range(2)]
        self._pinned = {}  # pair -> host buffers (keep_all)
        self._done = [None, None]  # copy-stream event of the last host copy out of each staging slot
        self._cur = -1
        self.d2h_events = []  # (start, end, bytes) per chunk on the copy stream
        self.pairs = 0
        self._width = {}  # pair -> samples per line (the first pair's K + 1, later pairs K)
        self._slot_pair = [None, None]  # the pair whose lines each buffer slot holds

    def _bufs(self, dev):
        t = self.torch
        pin = dict(pin_memory=True) if dev == "cpu" else {}
        return dict(points=t.empty((self.n, self.P, 3), dtype=t.float64, device=dev, **pin),
                    velocity=t.empty((self.n, self.P, 3), dtype=t.float64, device=dev, **pin),
                    temperature=t.empty((self.n, self.P), dtype=t.float64, device=dev, **pin),
                    salinity=t.empty((self.n, self.P), dtype=t.float64, device=dev, **pin),
                    ids=t.empty((self.n,), dtype=t.int32, device=dev, **pin))

    def host(self, p: int) -> dict:
        """Pair p's lines on the host (rows in the chain's slot order, ``ids`` = each row's particle)."""
        if not self.keep_all and self._slot_pair[p % 2] != p:
            raise ValueError(f"pair {p}'s host lines were overwritten by pair {self._slot_pair[p % 2]} (keep_all=False "
                             "holds the last two pairs)")
        b = self._pinned[p] if self.keep_all else self.hostbufs[p % 2]
        w = self._width[p]
        return {k: (v if k == "ids" else v[:, :w]) for k, v in b.items()}

    def __call__(self, p: int, lines: dict, ids):
        torch = self.torch
        cs = torch.cuda.current_stream(self.dev)
        slot = p % 2
        if p != self._cur:  # first chunk of pair p: slot p % 2's previous host copy must be done
            self._cur, self._row = p, 0
            if self._done[slot] is not None:
                cs.wait_event(self._done[slot])
            self.pairs += 1
            self._slot_pair[slot] = p
            if self.keep_all:
                self._pinned[p] = self._bufs("cpu")
        w = lines["points"].shape[1]
        self._width[p] = w
        lo, hi = self._row, self._row + lines["points"].shape[0]
        if hi > self.n or w > self.P:
            raise ValueError(f"HostLineSink sized for {self.n} lines of {self.P} samples: pair {p} hands rows up to {hi} "
                             f"of {w} samples")
        self._row = hi
        st = self.stage[slot]
        for k, v in lines.items():  # compute stream: device staging (the chain reuses its chunk buffers next)
            st[k][lo:hi, :w].copy_(v)
        st["ids"][lo:hi].copy_(ids)
        ready = torch.cuda.Event()
        ready.record(cs)
        self.copy.wait_event(ready)
        dst = self._pinned[p] if self.keep_all else self.hostbufs[slot]
        with torch.cuda.stream(self.copy):
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(self.copy)
            nbytes = 0
            for k in ("points", "velocity", "temperature", "salinity"):
                # whole rows lo..hi of the staging slab (contiguous), the first w samples of each are the pair's
                dst[k][lo:hi].copy_(st[k][lo:hi], non_blocking=True)
                nbytes += st[k][lo:hi].numel() * 8
            dst["ids"][lo:hi].copy_(st["ids"][lo:hi], non_blocking=True)
            nbytes += (hi - lo) * 4
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(self.copy)
        self.d2h_events.append((e0, e1, nbytes))
        self._done[slot] = e1

    def synchronize(self):
        self.copy.synchronize()

    def d2h_stats(self) -> dict:
        """Bytes, milliseconds and GB/s of the host copies so far (copy-stream events; after synchronize)."""
        ms = sum(a.elapsed_time(b) for (a, b, _) in self.d2h_events)
        by = sum(n for (_, _, n) in self.d2h_events)
        return {"bytes": by, "ms": ms, "gbs": by / (ms * 1e-3) / 1e9 if ms > 0 else None,
                "chunks": len(self.d2h_events), "pairs": self.pairs}


def cu_split_streams(device, side_cus: int):
    """(compute, side): two HIP streams that partition the device's CUs
    (hipExtStreamCreateWithCUMask), ``side_cus`` of them for the side stream.
    The side CUs are bits k*(n_cu/side_cus + 1) mod n_cu, which put one on each
    XCD whether the mask's bits map to XCDs in contiguous blocks or round-robin
    (256 CUs, 8 side CUs: bits 0, 33, 66, ...).  The streams live until exit."""
    import ctypes as C
    import torch
    dev = torch.device(device)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    if not (0 < side_cus < n_cu):
        raise ValueError("side_cus must leave CUs on both sides")
    stride = n_cu // side_cus + 1
    side_bits = {(k * stride) % n_cu for k in range(side_cus)}
    if len(side_bits) != side_cus:
        side_bits = set(range(side_cus))
    words = (n_cu + 31) // 32
    lib = L.load()  # its hipExtStreamCreateWithCUMask is the HIP runtime torch uses (see _lib.load)
    lib.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
    lib.hipExtStreamCreateWithCUMask.restype = C.c_int
    out = []
    for mine in (lambda b: b not in side_bits, lambda b: b in side_bits):
        mask = (C.c_uint32 * words)()
        for b in range(n_cu):
            if mine(b):
                mask[b // 32] |= 1 << (b % 32)
        h = C.c_void_p()
        with torch.cuda.device(dev):
            rc = lib.hipExtStreamCreateWithCUMask(C.byref(h), words, mask)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
        out.append(torch.cuda.ExternalStream(h.value, device=dev))
    return out[0], out[1]


def snapshot_field_factory(mesh: DeviceMesh, make_snapshot):
    """``make_field`` for PathlineChain from a host ``make_snapshot(i)`` (raw MPASOSolution arrays)."""
    def make(i, stream):
        return DeviceField.from_snapshot(mesh, make_snapshot(i), stream=stream)
    return make
