"""Synthetic snapshot fields generated directly in HBM.

Same analytic flow as :func:`mops_amd.synth.make_snapshot` (solid body +
travelling wave-3, depth decay, w on the interface grid), evaluated on the GPU
by one HIP kernel (mops_amd/csrc/mops_synth.hip -> lib/libmops_synth.so), so
long pathline chains on oRRS18to6-class meshes (3.5M cells x
80 levels: 2.2 GB per raw field) can stream dozens of daily snapshots through
``mops_field_create_device`` without building them on the host.  Values agree
with the numpy generator to rounding (libm vs device sin/cos); the parity
tests use the numpy generator, this module only feeds the configs 4/5 bench.
"""
from __future__ import annotations

import numpy as np


class DeviceSnapshotSource:
    """Per-mesh constants on the device; ``make(timestep, phase)`` returns the raw
    MPASOSolution arrays of one snapshot as float64 CUDA tensors."""

    def __init__(self, mesh, device, u0: float = 0.5, u1: float = 0.25, w0: float = 1.0e-5):
        import torch
        self.torch = torch
        self.device = device
        self.L = int(mesh.nVertLevels)
        self.lat = torch.as_tensor(np.ascontiguousarray(mesh.lat_cell, dtype=np.float64), device=device)
        self.lon = torch.as_tensor(np.ascontiguousarray(mesh.lon_cell, dtype=np.float64), device=device)
        rbd = np.asarray(mesh.refBottomDepth, dtype=np.float64)
        self.H = float(rbd[-1])
        self.ref_dz = torch.as_tensor(np.diff(np.concatenate([[0.0], rbd])), device=device)
        self.u0, self.u1, self.w0 = u0, u1, w0

    def make(self, timestep: int = 0, phase: float = 0.0) -> dict:
        """One snapshot's raw arrays, generated on the current stream by libmops_synth.so
        (mops_amd/csrc/mops_synth.hip: one pass per cell)."""
        import ctypes as C
        torch = self.torch
        n, L, dev = int(self.lat.shape[0]), self.L, self.device
        out = {k: torch.empty(shape, dtype=torch.float64, device=dev) for k, shape in
               (("layerThickness", (n, L)), ("bottomDepth", (n,)), ("zonalVelocity", (n, L)),
                ("meridionalVelocity", (n, L)), ("vertVelocityTop", (n, L + 1)))}
        P = C.c_void_p
        rc = _synth_lib().mops_synth_snapshot(
            C.c_int64(n), C.c_int(L), P(self.lat.data_ptr()), P(self.lon.data_ptr()), P(self.ref_dz.data_ptr()),
            C.c_double(self.H), C.c_double(phase), C.c_double(self.u0), C.c_double(self.u1), C.c_double(self.w0),
            P(out["layerThickness"].data_ptr()), P(out["bottomDepth"].data_ptr()), P(out["zonalVelocity"].data_ptr()),
            P(out["meridionalVelocity"].data_ptr()), P(out["vertVelocityTop"].data_ptr()),
            P(torch.cuda.current_stream(dev).cuda_stream))
        if rc != 0:
            raise RuntimeError("mops_synth_snapshot failed")
        out["timestep"] = int(timestep)
        return out


_SYNTH = None


def _synth_lib():
    """libmops_synth.so (built in-tree by __graft_entry__.build_synth)."""
    global _SYNTH
    if _SYNTH is None:
        import ctypes
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libmops_synth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run __graft_entry__.build()")
        _SYNTH = ctypes.CDLL(path)
    return _SYNTH


class DeviceFieldRecycler:
    """``make_field`` for :class:`mops_amd.chain.PathlineChain` with in-place refills.

    * ``self(i, stream)`` creates a field (chain start: snapshots 0 and 1);
    * ``prepare(i)`` generates snapshot i's raw arrays on a side stream, so it
      overlaps the running pair (one raw set, reused once its last reader is done);
    * ``refill(field, i, stream)`` re-derives the finished pair's field in place
      from them (mops_field_rebuild_device): no allocation, no host sync;
    * ``release(field)`` keeps a field the chain no longer needs for the next
      ``self(i, stream)``, which then re-derives it instead of allocating (field
      buffers are ~75 GB on an oRRS18to6-class mesh: their hipMalloc is setup,
      not per-run work).
    """

    def __init__(self, dmesh, source: DeviceSnapshotSource, phase_per_snapshot: float = 0.35):
        torch = source.torch
        self.torch = torch
        self.dmesh = dmesh
        self.source = source
        self.phase = phase_per_snapshot
        self.side = torch.cuda.Stream(device=source.device)
        self.raw = None
        self.raw_i = None
        self.ready = None
        self.consumed = None
        self.pool = []

    def release(self, field):
        self.pool.append(field)

    def __call__(self, i, stream):
        from .engine import DeviceField
        torch = self.torch
        if self.pool:
            ts = torch.cuda.ExternalStream(stream) if isinstance(stream, int) and stream else \
                torch.cuda.current_stream(self.source.device)
            return self.refill(self.pool.pop(), i, ts)
        snap = self.source.make(timestep=i, phase=self.phase * i)
        torch.cuda.current_stream(self.source.device).synchronize()
        f = DeviceField.from_device_snapshot(self.dmesh, snap, timestep=i, stream=stream)
        del snap
        return f

    def prepare(self, i, after=None):
        """``after``: an event the generation also waits for (the chain passes one recorded right before
        a trajectory launch, so the generation runs beside that launch instead of in front of the
        small kernels that precede it)."""
        torch = self.torch
        with torch.cuda.stream(self.side):
            if self.consumed is not None:
                self.side.wait_event(self.consumed)  # the previous refill has read the raw set
            if after is not None:
                self.side.wait_event(after)
            self.raw = None
            self.raw = self.source.make(timestep=i, phase=self.phase * i)
            self.ready = torch.cuda.Event()
            self.ready.record(self.side)
            self.raw_i = i

    def refill(self, field, i, stream):
        """``stream``: the torch stream the chain computes on."""
        torch = self.torch
        if self.raw_i != i:
            self.prepare(i)
        stream.wait_event(self.ready)
        field.rebuild_from_device(self.raw, timestep=i, stream=stream.cuda_stream)
        self.consumed = torch.cuda.Event()
        self.consumed.record(stream)
        return field


def device_field_factory(dmesh, source: DeviceSnapshotSource, phase_per_snapshot: float = 0.35):
    """Plain ``make_field(i, stream)``: snapshot i generated and derived in HBM into a new field."""
    from .engine import DeviceField
    torch = source.torch

    def make(i, stream):
        snap = source.make(timestep=i, phase=phase_per_snapshot * i)
        torch.cuda.current_stream(source.device).synchronize()  # generated before the engine reads it
        f = DeviceField.from_device_snapshot(dmesh, snap, timestep=i, stream=stream)
        del snap  # mops_field_create_device synchronises its stream before returning
        torch.cuda.empty_cache()  # hand the raw-field blocks back: the engine allocates fields with hipMalloc
        return f
    return make
