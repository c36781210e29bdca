"""Device-resident trajectory engine: thin owner objects over the C ABI.

``DeviceMesh`` / ``DeviceField`` keep the mesh and derived snapshots resident
in HBM (uploaded once, unlike the reference's HIP backend which re-uploads
every array per call, src/GPU/HIP/Kernel/MPASOVisualizerKernels.cu:1369-1431).
``ParticleSet`` is the SoA particle state + record slab as torch tensors
(torch is plumbing: allocation and streams), driven segment by segment by
``advance`` so records can be gathered while the next segment computes.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import dataclasses

import numpy as np

from . import _lib as L


def _nullcontext():
    return contextlib.nullcontext()


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _stream_handle(stream) -> C.c_void_p:
    if stream is None:
        return C.c_void_p(0)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(int(stream.cuda_stream))


@dataclasses.dataclass
class TrajectoryConfig:
    """TrajectorySettings (src/Core/MPASOVisualizer.h:90-103)."""
    deltaT: int = 120
    simulationDuration: int = 86400
    recordT: int = 3600
    depth: float = 0.0
    direction: int = L.MOPS_FORWARD
    method: int = L.MOPS_EULER          # reference default (MPASOVisualizer.h:99)

    def ctype(self) -> L.TrajCfg:
        return L.TrajCfg(int(self.deltaT), int(self.simulationDuration), int(self.recordT), int(self.direction),
                         int(self.method))

    @property
    def n_records(self) -> int:
        return int(self.simulationDuration // self.recordT) if self.recordT > 0 else 0

    @property
    def n_steps(self) -> int:
        return int(self.simulationDuration // self.deltaT) if self.deltaT > 0 else 0


class DeviceMesh:
    """MPAS-O mesh resident on the current HIP device (mops_mesh_create)."""

    def __init__(self, *, nCells, nVertices, maxEdges, nVertLevels, nEdgesOnCell, verticesOnCell, cellsOnCell,
                 cellsOnVertex, cellCoord, vertexCoord, stream=None):
        lib = L.load()
        self._arrays = dict(
            ne=np.ascontiguousarray(nEdgesOnCell, dtype=np.uint64),
            voc=np.ascontiguousarray(verticesOnCell, dtype=np.uint64),
            coc=np.ascontiguousarray(cellsOnCell, dtype=np.uint64),
            cov=None if cellsOnVertex is None else np.ascontiguousarray(cellsOnVertex, dtype=np.uint64),
            cc=np.ascontiguousarray(cellCoord, dtype=np.float64).reshape(-1),
            vc=np.ascontiguousarray(vertexCoord, dtype=np.float64).reshape(-1))
        a = self._arrays
        desc = L.MeshDesc(int(nCells), int(nVertices), int(maxEdges), int(nVertLevels), _ptr(a["ne"]), _ptr(a["voc"]),
                          _ptr(a["coc"]), _ptr(a["cov"]), _ptr(a["cc"]), _ptr(a["vc"]))
        h = C.c_void_p()
        L.check(lib.mops_mesh_create(C.byref(desc), _stream_handle(stream), C.byref(h)), "mops_mesh_create")
        self.handle = h
        self.nCells, self.nVertices, self.maxEdges, self.nVertLevels = int(nCells), int(nVertices), int(maxEdges), \
            int(nVertLevels)
        self._arrays = None  # the library copied everything

    @classmethod
    def from_mesh(cls, m, stream=None):
        return cls(nCells=m.nCells, nVertices=m.nVertices, maxEdges=m.maxEdges, nVertLevels=m.nVertLevels,
                   nEdgesOnCell=m.nEdgesOnCell, verticesOnCell=m.verticesOnCell, cellsOnCell=m.cellsOnCell,
                   cellsOnVertex=m.cellsOnVertex, cellCoord=m.cellCoord, vertexCoord=m.vertexCoord, stream=stream)

    def set_edges(self, nEdges, edgesOnCell, cellsOnEdge, edgeCoord, stream=None):
        """Upload the mesh's edges for the RBF velocity reconstruction (mops_mesh_set_edges)."""
        eoc = np.ascontiguousarray(edgesOnCell, dtype=np.uint64)
        coe = np.ascontiguousarray(cellsOnEdge, dtype=np.uint64)
        ec = np.ascontiguousarray(edgeCoord, dtype=np.float64).reshape(-1)
        L.check(L.load().mops_mesh_set_edges(self.handle, int(nEdges), _ptr(eoc), _ptr(coe), _ptr(ec),
                                             _stream_handle(stream)), "mops_mesh_set_edges")
        self.nEdges = int(nEdges)
        return self

    @property
    def nbytes(self) -> int:
        return int(L.load().mops_mesh_bytes(self.handle))

    def locate(self, d_points, d_cells, n: int, stream=None, d_hint=None):
        """Device pointers (ints) -> nearest cell ids (mops_locate_cells; with a
        candidate cell per point, mops_locate_cells_hinted -- same answer)."""
        if d_hint is None:
            L.check(L.load().mops_locate_cells(self.handle, n, C.c_void_p(d_points), C.c_void_p(d_cells),
                                               _stream_handle(stream)), "mops_locate_cells")
        else:
            L.check(L.load().mops_locate_cells_hinted(self.handle, n, C.c_void_p(d_points), C.c_void_p(d_hint),
                                                      C.c_void_p(d_cells), _stream_handle(stream)),
                    "mops_locate_cells_hinted")

    def close(self):
        if getattr(self, "handle", None):
            L.load().mops_mesh_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceField:
    """One derived snapshot resident in HBM (mops_field_create[_derived])."""

    def __init__(self, mesh: DeviceMesh, handle):
        self.mesh = mesh
        self.handle = handle

    @classmethod
    def from_snapshot(cls, mesh: DeviceMesh, snap, stream=None, velocity: str = "zonal"):
        """``velocity``: "zonal" -- the cell velocity from zonal/meridional components (the reference's
        live path, MOPSApp.cpp:113); "rbf" -- reconstructed from ``snap.normalVelocity`` on the edges
        (MPASOSolution::calcCellCenterVelocity; the mesh needs ``DeviceMesh.set_edges``)."""
        lib = L.load()
        rbf = velocity == "rbf"
        keep = [np.ascontiguousarray(x, dtype=np.float64) if x is not None else None for x in
                (snap.layerThickness, snap.bottomDepth, getattr(snap, "surfaceHeight", None),
                 None if rbf else snap.zonalVelocity, None if rbf else snap.meridionalVelocity, snap.vertVelocityTop,
                 getattr(snap, "normalVelocity", None) if rbf else None)]
        desc = L.SnapshotDesc(int(snap.timestep), *[_ptr(x) for x in keep])
        h = C.c_void_p()
        L.check(lib.mops_field_create(mesh.handle, C.byref(desc), _stream_handle(stream), C.byref(h)),
                "mops_field_create")
        return cls(mesh, h)

    @staticmethod
    def _device_desc(snap: dict, timestep: int):
        def dp(k):
            t = snap.get(k)
            if t is None:
                return None
            if not (t.is_cuda and t.dtype.is_floating_point and t.element_size() == 8 and t.is_contiguous()):
                raise ValueError(f"{k}: expected a contiguous float64 CUDA tensor")
            return C.c_void_p(t.data_ptr())
        return L.SnapshotDesc(int(timestep), dp("layerThickness"), dp("bottomDepth"), dp("surfaceHeight"),
                              dp("zonalVelocity"), dp("meridionalVelocity"), dp("vertVelocityTop"),
                              dp("normalVelocity"))

    @classmethod
    def from_device_snapshot(cls, mesh: DeviceMesh, snap: dict, timestep: int = 0, stream=None):
        """Raw fields already in HBM (float64 CUDA tensors keyed like synth.Snapshot:
        layerThickness, bottomDepth, zonalVelocity, meridionalVelocity, vertVelocityTop;
        optional surfaceHeight) -- mops_field_create_device, no host round trip.
        Synchronises ``stream`` before returning."""
        desc = cls._device_desc(snap, timestep)
        h = C.c_void_p()
        L.check(L.load().mops_field_create_device(mesh.handle, C.byref(desc), _stream_handle(stream), C.byref(h)),
                "mops_field_create_device")
        return cls(mesh, h)

    def rebuild_from_device(self, snap: dict, timestep: int = 0, stream=None):
        """Re-derive this field in place from another snapshot's HBM tensors
        (mops_field_rebuild_device): asynchronous on ``stream``, stream-ordered
        after every earlier launch that reads this field there."""
        desc = self._device_desc(snap, timestep)
        L.check(L.load().mops_field_rebuild_device(self.handle, C.byref(desc), _stream_handle(stream)),
                "mops_field_rebuild_device")
        return self

    @classmethod
    def from_derived(cls, mesh: DeviceMesh, vertex_ztop, vertex_vel, vertex_w=None, stream=None):
        lib = L.load()
        zt = np.ascontiguousarray(vertex_ztop, dtype=np.float64)
        ve = np.ascontiguousarray(vertex_vel, dtype=np.float64)
        w = None if vertex_w is None else np.ascontiguousarray(vertex_w, dtype=np.float64)
        h = C.c_void_p()
        L.check(lib.mops_field_create_derived(mesh.handle, _ptr(zt), _ptr(ve), _ptr(w), _stream_handle(stream),
                                              C.byref(h)), "mops_field_create_derived")
        return cls(mesh, h)

    def export(self, stream=None):
        V, Lv = self.mesh.nVertices, self.mesh.nVertLevels
        zt = np.empty(V * Lv); ve = np.empty(V * Lv * 3); w = np.empty(V * (Lv + 1))
        L.check(L.load().mops_field_export(self.handle, _ptr(zt), _ptr(ve), _ptr(w), _stream_handle(stream)),
                "mops_field_export")
        return zt, ve, w

    @property
    def nbytes(self) -> int:
        return int(L.load().mops_field_bytes(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            L.load().mops_field_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_trajectories(mesh: DeviceMesh, front: DeviceField, back: DeviceField | None, cfg: TrajectoryConfig,
                     seeds: np.ndarray, depths: np.ndarray | None = None, cells: np.ndarray | None = None,
                     stream=None):
    """Host-in/host-out StreamLine (back None) or PathLine (mops_run_trajectories).

    Returns a dict of numpy arrays shaped like the reference's finalized
    lines: points/velocity [N, K+1, 3], temperature/salinity [N, K+1],
    lastPoint [N, 3], plus final_pos, final_depth, death_step, cells.
    """
    lib = L.load()
    seeds = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 3)
    n = seeds.shape[0]
    K = cfg.n_records
    P = K + 1
    out = dict(points=np.empty((n, P, 3)), velocity=np.empty((n, P, 3)), temperature=np.empty((n, P)),
               salinity=np.empty((n, P)), lastPoint=np.empty((n, 3)), final_pos=np.empty((n, 3)),
               final_depth=np.empty(n, dtype=np.float32), death_step=np.empty(n, dtype=np.int32))
    dep = None if depths is None else np.ascontiguousarray(depths, dtype=np.float32)
    cl = np.full(n, -1, dtype=np.int32) if cells is None else np.ascontiguousarray(cells, dtype=np.int32).copy()
    c = cfg.ctype()
    st = lib.mops_run_trajectories(mesh.handle, front.handle, None if back is None else back.handle, C.byref(c), n,
                                   _ptr(seeds), _ptr(dep), C.c_float(cfg.depth), _ptr(cl), _ptr(out["points"]),
                                   _ptr(out["velocity"]), _ptr(out["temperature"]), _ptr(out["salinity"]),
                                   _ptr(out["lastPoint"]), _ptr(out["final_pos"]), _ptr(out["final_depth"]),
                                   _ptr(out["death_step"]), _stream_handle(stream))
    L.check(st, "mops_run_trajectories")
    out["cells"] = cl
    return out


class ParticleSet:
    """Device-resident SoA particle state + [K][6][n] record slab (torch tensors).

    This is the bench / multi-GPU driver: inputs stay in HBM, ``advance``
    launches the trajectory kernel over a step range on a given stream.
    """

    def __init__(self, mesh: DeviceMesh, seeds_xyz, depth: float | np.ndarray, cfg: TrajectoryConfig, device=None,
                 cells=None, use_order: bool = True, record_stride: int | None = None):
        """``record_stride``: columns of the [K][6][stride] record slab (default n); a multi-GPU
        shard pads it to the largest shard so every rank's slab has one shape
        (distributed.RecordGather)."""
        import torch
        self.use_order = use_order
        self.torch = torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        if isinstance(seeds_xyz, torch.Tensor):  # already resident: no host round trip
            s = seeds_xyz.to(device=dev, dtype=torch.float64).reshape(-1, 3).clone()
        else:
            s = torch.as_tensor(np.ascontiguousarray(seeds_xyz, dtype=np.float64).reshape(-1, 3), device=dev)
        self.n = int(s.shape[0])
        self.mesh = mesh
        self.cfg = cfg
        self.seeds = s.contiguous()
        self.x = s[:, 0].contiguous(); self.y = s[:, 1].contiguous(); self.z = s[:, 2].contiguous()
        if np.isscalar(depth):
            self.depth = torch.full((self.n,), float(depth), dtype=torch.float32, device=dev)
        else:
            self.depth = torch.as_tensor(np.asarray(depth, dtype=np.float32), device=dev).contiguous()
        self.death = torch.full((self.n,), -1, dtype=torch.int32, device=dev)
        if cells is None:
            self.cell = torch.empty((self.n,), dtype=torch.int32, device=dev)
            mesh.locate(self.seeds.data_ptr(), self.cell.data_ptr(), self.n,
                        stream=torch.cuda.current_stream(dev).cuda_stream)
        else:
            self.cell = torch.as_tensor(np.asarray(cells, dtype=np.int32), device=dev).contiguous()
        self.K = cfg.n_records
        self.rec_stride = self.n if record_stride is None else int(record_stride)
        if self.rec_stride < self.n:
            raise ValueError("record_stride below the particle count")
        self.records = torch.zeros((max(self.K, 1), 6, self.rec_stride), dtype=torch.float64, device=dev)
        self.order = torch.empty((self.n,), dtype=torch.int32, device=dev)
        # slot -> particle index: with use_order the state is kept PHYSICALLY in
        # locality order (state loads/stores and record stores coalesce);
        # finalize() writes line ids[slot], so outputs keep the seed order
        self.ids = torch.arange(self.n, dtype=torch.int32, device=dev)
        self._compact_scratch = {}
        self._spare = {}  # second buffers for the permutations (_apply_order)
        self._n_live = {}  # (lo, hi) -> device int32: live particles at the front of the range after compact()
        self._written = False
        self._c = cfg.ctype()
        self.reorder(stream=torch.cuda.current_stream(dev).cuda_stream)

    def reorder(self, stream=None, records_written: int | None = None):
        """Locality order of the particles by their current cell (mops_order_particles), applied by permuting
        the SoA state (and the records once written: every slot -- a particle that died already holds
        the reference's zeros in its later slots -- or the first ``records_written`` when no particle can
        have died yet) so slot s holds particle ids[s]."""
        L.check(L.load().mops_order_particles(self.mesh.handle, self.n, C.c_void_p(self.cell.data_ptr()),
                                              C.c_void_p(self.order.data_ptr()), _stream_handle(stream)),
                "mops_order_particles")
        if not self.use_order or self.n == 0:
            return
        slots = self.records.shape[0] if self._written else 0
        if records_written is not None:
            slots = min(slots, max(0, int(records_written)))
        self._apply_order(self.order, 0, self.n, stream, slots)

    _STATE = (("x", 8), ("y", 8), ("z", 8), ("depth", 4), ("cell", 4), ("death", 4), ("ids", 4), ("seeds", 24))

    def _apply_order(self, order, lo: int, hi: int, stream, record_slots: int):
        """Permute slots [lo, hi) of the SoA state, seeds, slot ids and the first ``record_slots`` record
        slots by ``order`` (local indices) with one mops_permute_arrays launch into the spare buffers;
        the whole set swaps buffers, a sub-range is copied back with a second launch."""
        torch = self.torch
        n = hi - lo
        if n <= 0:
            return
        if isinstance(stream, int):
            s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream(self.seeds.device)
        else:
            s = stream if stream is not None else torch.cuda.current_stream(self.seeds.device)
        names = [(k, e) for k, e in self._STATE] + ([("records", 8)] if record_slots > 0 else [])
        with torch.cuda.stream(s):
            for k, _ in names:
                if k not in self._spare:  # (allocated on first use, then kept)
                    self._spare[k] = torch.empty_like(getattr(self, k))

        def desc(src, dst, name, eb):
            if name == "records":
                return L.PermArray(src.data_ptr() + 8 * lo, dst.data_ptr() + 8 * lo, 8, int(record_slots) * 6,
                                   self.rec_stride)
            return L.PermArray(src.data_ptr() + eb * lo, dst.data_ptr() + eb * lo, eb, 1, n)

        lib = L.load()
        arr = (L.PermArray * len(names))(*[desc(getattr(self, k), self._spare[k], k, e) for k, e in names])
        L.check(lib.mops_permute_arrays(n, C.c_void_p(order.data_ptr() + 4 * lo), len(names), arr, _stream_handle(s)),
                "mops_permute_arrays")
        if lo == 0 and hi == self.n:
            for k, _ in names:  # the gathered copies become the state
                cur = getattr(self, k)
                setattr(self, k, self._spare[k])
                self._spare[k] = cur
        else:
            back = (L.PermArray * len(names))(*[desc(self._spare[k], getattr(self, k), k, e) for k, e in names])
            L.check(lib.mops_permute_arrays(n, None, len(names), back, _stream_handle(s)), "mops_permute_arrays")

    def original(self, t):
        """A per-slot tensor back in the particles' seed order."""
        out = self.torch.empty_like(t)
        out[self.ids.long()] = t
        return out

    def compact(self, lo: int, hi: int, stream, records_written: int):
        """Dead-particle compaction of slots [lo, hi) on ``stream`` (mops_order_particles_live):
        live particles in the Morton order of their current cell first, dead ones after them, so
        the next launches run full waves of live lanes and all-dead waves exit at once.  The SoA
        state, seeds, slot ids and the first ``records_written`` record slots are permuted with
        them; the dead particles' later slots are cleared again where they land
        (mops_records_clear_dead: they hold no samples, the live particles' ones are written by
        the next launches).  Results are unchanged (every particle is independent, finalize
        writes each slot's line at its id).  Re-entrant across disjoint ranges on different
        streams (each range has its own scratch)."""
        torch = self.torch
        n = hi - lo
        if n <= 1:
            return
        lib = L.load()
        s = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.ExternalStream(int(stream))
        key = (lo, hi)
        if key not in self._compact_scratch:
            nb = int(lib.mops_order_scratch_bytes(n))
            if nb <= 0:
                raise L.MopsError("mops_order_scratch_bytes failed")
            with torch.cuda.stream(s):
                self._compact_scratch[key] = torch.empty((nb,), dtype=torch.uint8, device=self.seeds.device)
        scratch = self._compact_scratch[key]
        if key not in self._n_live:
            with torch.cuda.stream(s):
                self._n_live[key] = torch.zeros((1,), dtype=torch.int32, device=self.seeds.device)
        e4 = 4
        L.check(lib.mops_order_particles_live(self.mesh.handle, n, C.c_void_p(self.cell.data_ptr() + e4 * lo),
                                              C.c_void_p(self.death.data_ptr() + e4 * lo),
                                              C.c_void_p(self.order.data_ptr() + e4 * lo),
                                              C.c_void_p(self._n_live[key].data_ptr()),
                                              C.c_void_p(scratch.data_ptr()), scratch.numel(), _stream_handle(s)),
                "mops_order_particles_live")
        kw = min(int(records_written), self.records.shape[0])
        self._apply_order(self.order, lo, hi, s, kw)
        L.check(lib.mops_records_clear_dead(n, C.c_void_p(self._n_live[key].data_ptr()), kw, self.K,
                                            C.c_void_p(self.records.data_ptr() + 8 * lo), self.rec_stride,
                                            _stream_handle(s)), "mops_records_clear_dead")
        return self._n_live[key]

    def set_config(self, cfg: TrajectoryConfig):
        """Run the next call with ``cfg`` (a chained pair's own simulationDuration: its step and
        record counts and alpha ramp); its records must fit the slab allocated at creation."""
        if cfg.n_records > self.records.shape[0]:
            raise ValueError(f"{cfg.n_records} records do not fit the slab of {self.records.shape[0]}")
        self.cfg = cfg
        self._c = cfg.ctype()
        self.K = cfg.n_records

    def swap_records(self, slab):
        """Install another [K][6][stride] slab as the record buffer and return the current one
        (RecordGather: the slab just completed is gathered while the next call writes this one)."""
        if tuple(slab.shape) != tuple(self.records.shape) or slab.dtype != self.records.dtype:
            raise ValueError("record slab shape/dtype mismatch")
        old, self.records = self.records, slab
        return old

    def reset(self, depth=None):
        self.x.copy_(self.seeds[:, 0]); self.y.copy_(self.seeds[:, 1]); self.z.copy_(self.seeds[:, 2])
        if depth is not None:
            self.depth.fill_(float(depth))
        self.death.fill_(-1)
        self._written = False  # (records: every slot is rewritten by the launches from step 0)

    def reseed(self, seeds, depth, stream=None, hint_cells: bool = False):
        """Start a new run from device-resident seeds [n,3] (f64) and depth (scalar
        or [n] f32): state <- seeds, death cleared (records need no clearing), seed cells
        located (the reference's calcInWhichCells per run) and re-ordered.
        ``hint_cells``: the seeds continue this set's particles (a chained pair),
        so each particle's current cell seeds the exact locate (same answer)."""
        torch = self.torch
        s = seeds.reshape(-1, 3)
        if int(s.shape[0]) != self.n:
            raise ValueError("reseed: particle count changed")
        h = stream if stream is not None else torch.cuda.current_stream(self.seeds.device).cuda_stream
        # slot order -> particle order, before the ids reset (same stream as the copies below)
        hint = self.original(self.cell) if hint_cells else None
        self.seeds.copy_(s)
        self.ids.copy_(torch.arange(self.n, dtype=torch.int32, device=self.ids.device))
        self.x.copy_(s[:, 0]); self.y.copy_(s[:, 1]); self.z.copy_(s[:, 2])
        if isinstance(depth, torch.Tensor):
            self.depth.copy_(depth.to(torch.float32))
        else:
            self.depth.fill_(float(np.float32(depth)))
        self.death.fill_(-1)
        self._written = False
        self.mesh.locate(self.seeds.data_ptr(), self.cell.data_ptr(), self.n, stream=h,
                         d_hint=None if hint is None else hint.data_ptr())
        self.reorder(stream=h)

    def particles(self) -> L.Particles:
        return L.Particles(self.n, self.x.data_ptr(), self.y.data_ptr(), self.z.data_ptr(), self.depth.data_ptr(),
                           self.cell.data_ptr(), self.death.data_ptr(), None, None)  # physically ordered

    def advance(self, front: DeviceField, back: DeviceField | None, step_begin: int, step_end: int, stream=None,
                live_count=None):
        """Launch steps [step_begin, step_end) over every slot; ``live_count``: the device live count
        compact(0, n) returned (only the leading live slots are spread over the XCDs)."""
        p = self.particles() if live_count is None else self._sub_particles(0, self.n, live_count)
        st = L.load().mops_traj_advance(self.mesh.handle, front.handle, None if back is None else back.handle,
                                        C.byref(self._c), C.byref(p), int(step_begin), int(step_end),
                                        C.c_void_p(self.records.data_ptr()), self.rec_stride, _stream_handle(stream))
        L.check(st, "mops_traj_advance")
        self._written = True

    def _sub_particles(self, lo: int, hi: int, live_count=None) -> L.Particles:
        """Slots [lo, hi) as a launch argument; ``live_count``: the range's device live count after a
        compaction (only its leading live slots are launched over the XCDs)."""
        e4, e8 = 4, 8
        return L.Particles(hi - lo, self.x.data_ptr() + e8 * lo, self.y.data_ptr() + e8 * lo,
                           self.z.data_ptr() + e8 * lo, self.depth.data_ptr() + e4 * lo,
                           self.cell.data_ptr() + e4 * lo, self.death.data_ptr() + e4 * lo, None,
                           None if live_count is None else live_count.data_ptr())

    def advance_pipelined(self, front: DeviceField, back: DeviceField | None, step_begin: int, step_end: int,
                          streams, chunks: int, timing=None, compact: bool = False, compact_priority: bool = False):
        """``advance`` split into len(streams) contiguous particle parts (whole waves), each on its own
        stream, and ``chunks`` step ranges per part, enqueued chunk-major.

        One launch over all particles ends in a partial round of waves: 1e6 particles are 15625
        waves over 3072 resident slots (5.09 rounds), so the last 9% of a round runs alone for a
        whole wave lifetime.  Shorter launches on several streams let one part's tail overlap the
        other parts' next chunk (kernel boundaries order each part's chunks; results are
        identical for any split: every particle is independent and records are indexed by
        absolute step).  The streams must already be ordered after the state's producers; the
        caller joins them afterwards.  ``timing`` receives (start, end) events per launch.
        ``compact``: before every chunk but the first, each part is re-sorted on its own stream
        with its dead particles last (``compact``): RK4 kills particles at cell crossings
        (quirk Q1, half of them in a day at config 2), and a wave keeps its slots until its
        last live lane finishes."""
        torch = self.torch
        nparts = max(1, len(streams))
        pb = self.part_bounds(nparts)
        span = int(step_end) - int(step_begin)
        chunks = max(1, min(int(chunks), span))
        tb = [int(step_begin) + span * k // chunks for k in range(chunks + 1)]
        period = self.record_period(pathline=back is not None)
        lib = L.load()
        if compact and chunks > 1 and compact_priority:
            # optionally the re-sort runs on a high-priority stream per part: its short kernels otherwise
            # queue behind the other parts' trajectory waves (measured: the key kernel then waits ~5 ms)
            dev = self.seeds.device
            if getattr(self, "_hp_streams", None) is None or len(self._hp_streams) < nparts:
                prio = torch.cuda.Stream.priority_range()[1]  # the numerically lowest = highest priority
                self._hp_streams = [torch.cuda.Stream(device=dev, priority=prio) for _ in range(nparts)]
        for t in range(chunks):
            for k in range(nparts):
                lo, hi = pb[k], pb[k + 1]
                if hi <= lo or tb[t + 1] <= tb[t]:
                    continue
                st = streams[k]
                if compact and t > 0:
                    # slots written so far: slot 0 (step-0 pre-writes) .. the last completed record
                    nrec = min(self.K, tb[t] // period + 1) if period else 1
                    if compact_priority:
                        hp = self._hp_streams[k]
                        hp.wait_stream(st)
                        self.compact(lo, hi, hp, records_written=nrec)
                        st.wait_stream(hp)
                    else:
                        self.compact(lo, hi, st, records_written=nrec)
                if timing is not None:
                    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                p = self._sub_particles(lo, hi, self._n_live.get((lo, hi)) if (compact and t > 0) else None)
                rc = lib.mops_traj_advance(self.mesh.handle, front.handle, None if back is None else back.handle,
                                           C.byref(self._c), C.byref(p), tb[t], tb[t + 1],
                                           C.c_void_p(self.records.data_ptr() + 8 * lo), self.rec_stride,
                                           _stream_handle(st))
                L.check(rc, "mops_traj_advance")
                if timing is not None:
                    e1.record(st)
                    timing.append((e0, e1))
        self._written = True

    def part_bounds(self, nparts: int):
        """Slot bounds of ``nparts`` contiguous particle parts in whole waves (advance_pipelined)."""
        nparts = max(1, int(nparts))
        waves = -(-self.n // 64)
        return [min(self.n, 64 * (waves * k // nparts)) for k in range(nparts + 1)]

    def record_period(self, pathline: bool) -> int:
        import math
        if pathline:
            return int(self.cfg.recordT // self.cfg.deltaT)
        return int(self.cfg.recordT // math.gcd(int(self.cfg.recordT), int(self.cfg.deltaT)))

    def last_points(self, stream=None):
        """Each particle's cleaned last point in seed order (mops_traj_last_points): finalize's lastPoint
        without the lines."""
        torch = self.torch
        last = torch.empty((self.n, 3), dtype=torch.float64, device=self.seeds.device)
        L.check(L.load().mops_traj_last_points(self.n, self.K, C.c_void_p(self.seeds.data_ptr()),
                                               C.c_void_p(self.records.data_ptr()), self.rec_stride,
                                               C.c_void_p(self.ids.data_ptr()), C.c_void_p(last.data_ptr()),
                                               _stream_handle(stream)), "mops_traj_last_points")
        return last

    def finalize_from(self, seeds, ids, records, pathline: bool, stream=None):
        """finalize over another set's seeds, slot ids and record slab (a chain's deferred assembly: the
        buffers of a finished pair while this set runs the next)."""
        torch = self.torch
        dev = self.seeds.device
        P = self.K + 1
        pts = torch.empty((self.n, P, 3), dtype=torch.float64, device=dev)
        vel = torch.empty_like(pts)
        tmp = torch.empty((self.n, P), dtype=torch.float64, device=dev)
        sal = torch.empty_like(tmp)
        L.check(L.load().mops_traj_finalize(self.n, self.K, C.c_void_p(seeds.data_ptr()), C.c_void_p(records.data_ptr()),
                                            self.rec_stride, 1 if pathline else 0, C.c_void_p(ids.data_ptr()),
                                            C.c_void_p(pts.data_ptr()), C.c_void_p(vel.data_ptr()),
                                            C.c_void_p(tmp.data_ptr()), C.c_void_p(sal.data_ptr()), None,
                                            _stream_handle(stream)), "mops_traj_finalize")
        return dict(points=pts, velocity=vel, temperature=tmp, salinity=sal)

    def finalize_range(self, lo: int, hi: int, out: dict, pathline: bool, stream=None):
        """The lines of slots [lo, hi) into ``out`` (device tensors points [m, P, 3], velocity [m, P, 3],
        temperature / salinity [m, P], m = hi - lo) in slot order -- row i is particle ids[lo + i] -- a
        bounded piece of finalize (PathlineChain's writer hook)."""
        m = hi - lo
        if m <= 0:
            return out
        L.check(L.load().mops_traj_finalize(m, self.K, C.c_void_p(self.seeds.data_ptr() + 24 * lo),
                                            C.c_void_p(self.records.data_ptr() + 8 * lo), self.rec_stride,
                                            1 if pathline else 0, None, C.c_void_p(out["points"].data_ptr()),
                                            C.c_void_p(out["velocity"].data_ptr()),
                                            C.c_void_p(out["temperature"].data_ptr()),
                                            C.c_void_p(out["salinity"].data_ptr()), None, _stream_handle(stream)),
                "mops_traj_finalize")
        return out

    def finalize(self, pathline: bool, stream=None, streams=None, timing=None):
        """Lines of every particle in seed order (mops_traj_finalize).  ``streams``: the
        advance_pipelined part streams -- each part's lines are assembled on its own stream right
        after its last chunk, so one part's assembly overlaps the other parts' final waves (the
        caller joins the streams afterwards); ``timing`` receives (start, end) events per launch."""
        torch = self.torch
        dev = self.seeds.device
        P = self.K + 1
        pts = torch.empty((self.n, P, 3), dtype=torch.float64, device=dev)
        vel = torch.empty_like(pts)
        tmp = torch.empty((self.n, P), dtype=torch.float64, device=dev)
        sal = torch.empty_like(tmp)
        last = torch.empty((self.n, 3), dtype=torch.float64, device=dev)
        outs = (pts, vel, tmp, sal, last)
        if streams:
            pb = self.part_bounds(len(streams))
            parts = [(pb[k], pb[k + 1], streams[k]) for k in range(len(streams))]
            for t in outs:  # written on the part streams: the allocator must wait for them
                for st in streams:
                    t.record_stream(st if isinstance(st, torch.cuda.Stream) else torch.cuda.ExternalStream(int(st)))
        else:
            parts = [(0, self.n, stream)]
        lib = L.load()
        for lo, hi, st in parts:
            if hi <= lo:
                continue
            if timing is not None:
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                ts = st if isinstance(st, torch.cuda.Stream) else (
                    torch.cuda.ExternalStream(int(st)) if st else torch.cuda.default_stream(dev))
                e0.record(ts)
            # a part's slots write the lines ids[slot] of the full outputs
            rc = lib.mops_traj_finalize(hi - lo, self.K, C.c_void_p(self.seeds.data_ptr() + 24 * lo),
                                        C.c_void_p(self.records.data_ptr() + 8 * lo), self.rec_stride,
                                        1 if pathline else 0,
                                        C.c_void_p(self.ids.data_ptr() + 4 * lo), C.c_void_p(pts.data_ptr()),
                                        C.c_void_p(vel.data_ptr()), C.c_void_p(tmp.data_ptr()),
                                        C.c_void_p(sal.data_ptr()), C.c_void_p(last.data_ptr()), _stream_handle(st))
            L.check(rc, "mops_traj_finalize")
            if timing is not None:
                e1.record(ts)
                timing.append((e0, e1))
        return dict(points=pts, velocity=vel, temperature=tmp, salinity=sal, lastPoint=last)
