"""ctypes front-end of the CPU oracle (oracle/mops_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  The product (mops_amd) never
imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libmops_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "mops_oracle.c"))):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


class OrcMesh(C.Structure):
    _fields_ = [("n_cells", C.c_int64), ("n_vertices", C.c_int64), ("max_edges", C.c_int32),
                ("n_levels", C.c_int32), ("n_edges_on_cell", C.c_void_p), ("vertices_on_cell", C.c_void_p),
                ("cells_on_cell", C.c_void_p), ("cell_coord", C.c_void_p), ("vertex_coord", C.c_void_p)]


class OrcField(C.Structure):
    _fields_ = [("vertex_ztop", C.c_void_p), ("vertex_vel", C.c_void_p), ("vertex_w", C.c_void_p)]


class OrcCfg(C.Structure):
    _fields_ = [("delta_t", C.c_int64), ("duration", C.c_int64), ("record_t", C.c_int64),
                ("backward", C.c_int32), ("euler", C.c_int32)]


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        P = C.c_void_p
        _lib.orc_streamline.argtypes = [P, P, P, C.c_int64, P, P, P, P, P, P, P, C.c_int]
        _lib.orc_pathline.argtypes = [P, P, P, P, C.c_int64, P, P, P, P, P, P, P, C.c_int]
        _lib.orc_remove_nan.argtypes = [C.c_int64, P, P, P, P, P]
        _lib.orc_finalize.argtypes = [C.c_int64, C.c_int64, P, P, P, C.c_int, P, P, P, P, P]
        _lib.orc_cell_center_ztop.argtypes = [C.c_int64, C.c_int, P, P, P, P]
        _lib.orc_cell_to_vertex.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, P, P, P, P, P]
        _lib.orc_center_velocity_zm.argtypes = [C.c_int64, C.c_int, P, P, P, P]
        _lib.orc_knn.argtypes = [C.c_int64, P, C.c_int64, P, P, C.c_int]
        _lib.orc_gauss_elimination.argtypes = [P, P, C.c_int, P]
        _lib.orc_center_velocity_rbf.argtypes = [C.c_int64, C.c_int, C.c_int, P, P, P, P, P, P, P]
        _lib.orc_max_threads.restype = C.c_int
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class _Keep:
    """Holds numpy arrays alive for ctypes structs."""

    def __init__(self):
        self.refs = []

    def __call__(self, a, dtype):
        a = np.ascontiguousarray(a, dtype=dtype)
        self.refs.append(a)
        return a


def orc_mesh(mesh):
    k = _Keep()
    m = OrcMesh(mesh.nCells, mesh.nVertices, mesh.maxEdges, mesh.nVertLevels,
                _p(k(mesh.nEdgesOnCell, np.uint64)), _p(k(mesh.verticesOnCell, np.uint64)),
                _p(k(mesh.cellsOnCell, np.uint64)), _p(k(mesh.cellCoord, np.float64)),
                _p(k(mesh.vertexCoord, np.float64)))
    m._keep = k
    return m


class Derived:
    """Vertex fields the hot loop reads (cellVertexZTop/Velocity/VertVelocity)."""

    def __init__(self, vertex_ztop, vertex_vel, vertex_w, attrs=None):
        self.vertex_ztop = np.ascontiguousarray(vertex_ztop, dtype=np.float64)
        self.vertex_vel = np.ascontiguousarray(vertex_vel, dtype=np.float64)
        self.vertex_w = np.ascontiguousarray(vertex_w, dtype=np.float64)
        self.attrs = attrs or {}

    def orc(self):
        f = OrcField(_p(self.vertex_ztop), _p(self.vertex_vel), _p(self.vertex_w))
        f._keep = self
        return f


def center_velocity_rbf(mesh, normal_velocity):
    """TBBBackend::CalcCellCenterVelocity (MPASOSolutionTBB.cpp:131-245): cell-centre xyz velocity
    [C*L*3] from the edge-normal velocity [E*L] (the RBF path, no live caller in the reference)."""
    Cn, Lv = mesh.nCells, mesh.nVertLevels
    out = np.empty(Cn * Lv * 3)
    lib().orc_center_velocity_rbf(Cn, Lv, mesh.maxEdges,
                                  _p(np.ascontiguousarray(mesh.nEdgesOnCell, dtype=np.uint64)),
                                  _p(np.ascontiguousarray(mesh.edgesOnCell, dtype=np.uint64)),
                                  _p(np.ascontiguousarray(mesh.cellsOnEdge, dtype=np.uint64)),
                                  _p(np.ascontiguousarray(mesh.edgeCoord, dtype=np.float64)),
                                  _p(np.ascontiguousarray(mesh.cellCoord, dtype=np.float64)),
                                  _p(np.ascontiguousarray(normal_velocity, dtype=np.float64)), _p(out))
    return out


def preprocess(mesh, snap, velocity: str = "zonal") -> Derived:
    """MOPSApp::addSol derived fields (MOPSApp.cpp:100-129) via the oracle.  ``velocity``: "zonal"
    (CalcCellCenterVelocityByZM, the live path) or "rbf" (CalcCellCenterVelocity from
    snap.normalVelocity, MPASOSolution::calcCellCenterVelocity)."""
    L = lib()
    Cn, V, Lv = mesh.nCells, mesh.nVertices, mesh.nVertLevels
    cc = np.ascontiguousarray(mesh.cellCoord); vc = np.ascontiguousarray(mesh.vertexCoord)
    cov = np.ascontiguousarray(mesh.cellsOnVertex, dtype=np.uint64)
    ztc = np.empty(Cn * Lv)
    L.orc_cell_center_ztop(Cn, Lv, _p(snap.layerThickness), _p(snap.bottomDepth), None, _p(ztc))
    ztv = np.empty(V * Lv)
    L.orc_cell_to_vertex(Cn, V, Lv, 1, 0, _p(cov), _p(cc), _p(vc), _p(ztc), _p(ztv))
    if velocity == "rbf":
        velc = center_velocity_rbf(mesh, snap.normalVelocity)
    else:
        velc = np.empty(Cn * Lv * 3)
        L.orc_center_velocity_zm(Cn, Lv, _p(cc), _p(snap.zonalVelocity), _p(snap.meridionalVelocity), _p(velc))
    velv = np.empty(V * Lv * 3)
    L.orc_cell_to_vertex(Cn, V, Lv, 3, 0, _p(cov), _p(cc), _p(vc), _p(velc), _p(velv))
    wv = np.empty(V * (Lv + 1))
    L.orc_cell_to_vertex(Cn, V, Lv + 1, 1, 0, _p(cov), _p(cc), _p(vc), _p(snap.vertVelocityTop), _p(wv))
    attrs = {}
    for name in sorted(snap.attributes):
        av = np.empty(V * Lv)
        L.orc_cell_to_vertex(Cn, V, Lv, 1, 1, _p(cov), _p(cc), _p(vc), _p(snap.attributes[name]), _p(av))
        attrs[name] = av
    d = Derived(ztv, velv, wv, attrs)
    d.cell_ztop = ztc
    d.cell_vel = velc
    return d


def knn(mesh, pts, n_threads=0):
    out = np.empty(len(pts), dtype=np.int32)
    pts = np.ascontiguousarray(pts, dtype=np.float64)
    lib().orc_knn(mesh.nCells, _p(np.ascontiguousarray(mesh.cellCoord)), len(pts), _p(pts), _p(out),
                  n_threads or os.cpu_count())
    return out


def run(mesh, front: Derived, back, seeds, depth=0.0, depths=None, delta_t=120, duration=86400,
        record_t=3600, euler=True, backward=False, cells=None, n_threads=0, finalize=True):
    """Full StreamLine (back is None) / PathLine, reference semantics.

    Returns dict with the raw buffers, final state and (if finalize) the
    assembled lines exactly as FinalizeTrajectoryLines[WithAttrs] builds them.
    """
    L = lib()
    seeds = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 3)
    N = seeds.shape[0]
    K = duration // record_t
    if cells is None:
        cells = knn(mesh, seeds)
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    pts = seeds.copy()
    if depths is not None and len(depths) == N:
        dep = np.ascontiguousarray(depths, dtype=np.float32).copy()
    else:
        dep = np.full(N, np.float32(depth), dtype=np.float32)
    init_depth = dep.copy()
    rp = np.zeros(N * K * 3)
    rv = np.zeros(N * K * 3)
    death = np.empty(N, dtype=np.int32)
    last_cell = np.empty(N, dtype=np.int32)
    m = orc_mesh(mesh)
    cfg = OrcCfg(delta_t, duration, record_t, 1 if backward else 0, 1 if euler else 0)
    if back is None:
        rc = L.orc_streamline(C.byref(m), C.byref(front.orc()), C.byref(cfg), N, _p(pts), _p(dep), _p(cells),
                              _p(rp), _p(rv), _p(death), _p(last_cell), n_threads)
    else:
        rc = L.orc_pathline(C.byref(m), C.byref(front.orc()), C.byref(back.orc()), C.byref(cfg), N, _p(pts),
                            _p(dep), _p(cells), _p(rp), _p(rv), _p(death), _p(last_cell), n_threads)
    if rc != 0:
        return None
    out = dict(rec_pos=rp.reshape(N, K, 3), rec_vel=rv.reshape(N, K, 3), final_pos=pts, final_depth=dep,
               death=death, last_cell=last_cell, cells=cells, init_depth=init_depth)
    if finalize:
        out.update(finalize_lines(seeds, rp, rv, K, with_attrs=back is not None))
    return out


def finalize_lines(seeds, rec_pos, rec_vel, K, with_attrs):
    N = seeds.shape[0]
    P = K + 1
    points = np.empty((N, P, 3)); vel = np.empty((N, P, 3))
    temp = np.empty((N, P)); sal = np.empty((N, P)); last = np.empty((N, 3))
    lib().orc_finalize(N, K, _p(np.ascontiguousarray(seeds)), _p(np.ascontiguousarray(rec_pos)),
                       _p(np.ascontiguousarray(rec_vel)), 1 if with_attrs else 0, _p(points), _p(vel), _p(temp),
                       _p(sal), _p(last))
    return dict(points=points, velocity=vel, temperature=temp, salinity=sal, lastPoint=last)


def remove_nan(points, vel, temp, sal):
    points = np.ascontiguousarray(points, dtype=np.float64).copy()
    vel = np.ascontiguousarray(vel, dtype=np.float64).copy()
    temp = np.ascontiguousarray(temp, dtype=np.float64).copy()
    sal = np.ascontiguousarray(sal, dtype=np.float64).copy()
    last = np.empty(3)
    lib().orc_remove_nan(points.shape[0], _p(points), _p(vel), _p(temp), _p(sal), _p(last))
    return points, vel, temp, sal, last


def gauss_elimination(A, b):
    A = np.ascontiguousarray(A, dtype=np.float64).copy()
    b = np.ascontiguousarray(b, dtype=np.float64).copy()
    n = b.size
    x = np.zeros(n)
    lib().orc_gauss_elimination(_p(A), _p(b), n, _p(x))
    return x
