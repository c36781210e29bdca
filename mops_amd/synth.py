"""Synthetic MPAS-Ocean-like Voronoi meshes and snapshot fields.

No MPAS-Ocean mesh or history file exists offline, so every
parity test and benchmark runs on deterministic synthetic inputs of the same
shape as the reference's inputs:

* the mesh is the Voronoi dual of a frequency-``n`` icosahedral geodesic
  triangulation (``10 n^2 + 2`` cells: n=154 gives an EC30to60-class 237k-cell
  mesh, n=608 an oRRS18to6-class 3.7M-cell mesh), optionally culled by a land
  mask exactly the way MPAS culled ocean meshes look (missing neighbours are
  stored as id 0, boundary vertices carry a 0 in ``cellsOnVertex``);
* connectivity is emitted in the reference's own convention: ``size_t``
  (``uint64``) 1-based ``verticesOnCell``/``cellsOnCell`` of width
  ``maxEdges`` (zero padded), ``cellsOnVertex`` of width 3, xyz coordinates as
  ``vec3`` rows (``MPASOGrid`` members, reference ``src/Core/MPASOGrid.h``);
* a snapshot holds the raw per-cell fields ``MPASOSolution`` consumes in
  ``MOPSApp::addSol`` (``src/Core/MOPSApp.cpp:77-137``): layerThickness
  [C*L], bottomDepth [C], zonal/meridional velocity [C*L], vertical velocity
  [C*(L+1)] and two double attributes (temperature, salinity).

Everything is numpy-only and seeded, so a GPU box regenerates bit-identical
inputs without scipy.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

SPHERE_RADIUS = 6371229.0  # MPAS sphere_radius (m)
SEED_RADIUS = 6371010.0    # convertRadianLatLonToXYZ default r (GeoConverter.hpp:107, float literal)

_ICO_PHI = (1.0 + math.sqrt(5.0)) / 2.0


def _icosahedron():
    p = _ICO_PHI
    v = np.array([
        [-1, p, 0], [1, p, 0], [-1, -p, 0], [1, -p, 0],
        [0, -1, p], [0, 1, p], [0, -1, -p], [0, 1, -p],
        [p, 0, -1], [p, 0, 1], [-p, 0, -1], [-p, 0, 1]], dtype=np.float64)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    f = np.array([
        [0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11],
        [1, 5, 9], [5, 11, 4], [11, 10, 2], [10, 7, 6], [7, 1, 8],
        [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9],
        [4, 9, 5], [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=np.int64)
    return v, f


def geodesic_triangulation(n: int, jitter: float = 0.0, seed: int = 0):
    """Frequency-n geodesic triangulation of the unit sphere.

    Returns (points[P,3], triangles[T,3]) with every triangle counter-clockwise
    seen from outside.  ``jitter`` displaces points by that fraction of the
    mean spacing (keeps the mesh irregular like an SCVT, breaks symmetric ties).
    """
    if n < 1:
        raise ValueError("frequency must be >= 1")
    V, F = _icosahedron()
    # lattice (i, j) with i + j <= n on each face: point = A + i/n (B-A) + j/n (C-A)
    ii, jj = np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij")
    mask = ii + jj <= n
    ii, jj = ii[mask], jj[mask]
    nloc = ii.size
    A, B, C = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    pts = (A[:, None, :] + (ii[None, :, None] / n) * (B - A)[:, None, :]
           + (jj[None, :, None] / n) * (C - A)[:, None, :]).reshape(-1, 3)
    pts /= np.linalg.norm(pts, axis=1, keepdims=True)
    # dedup shared edge/corner points
    key = np.round(pts * 2.0**30).astype(np.int64)
    _, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    inv = inv.reshape(-1)
    # keep first-occurrence order so ids are deterministic
    order = np.argsort(first, kind="stable")
    remap = np.empty_like(order)
    remap[order] = np.arange(order.size)
    gid = remap[inv]
    uniq = pts[first[order]]
    # local lattice index lookup
    loc = -np.ones((n + 1, n + 1), dtype=np.int64)
    loc[ii, jj] = np.arange(nloc)
    tris = []
    for i in range(n):
        js = np.arange(0, n - i)
        a = loc[i, js]; b = loc[i + 1, js]; c = loc[i, js + 1]
        tris.append(np.stack([a, b, c], 1))
        if n - i - 1 > 0:
            js2 = np.arange(0, n - i - 1)
            a = loc[i + 1, js2]; b = loc[i + 1, js2 + 1]; c = loc[i, js2 + 1]
            tris.append(np.stack([a, b, c], 1))
    tl = np.concatenate(tris, 0)                       # [n^2, 3] local
    T = (tl[None, :, :] + (np.arange(20) * nloc)[:, None, None]).reshape(-1, 3)
    T = gid[T]
    if jitter > 0.0:
        rng = np.random.default_rng(seed)
        h = jitter * (1.1 / n)
        uniq = uniq + rng.normal(scale=h, size=uniq.shape)
        uniq /= np.linalg.norm(uniq, axis=1, keepdims=True)
    # orient CCW from outside
    a, b, c = uniq[T[:, 0]], uniq[T[:, 1]], uniq[T[:, 2]]
    nrm = np.cross(b - a, c - a)
    flip = np.einsum("ij,ij->i", nrm, a + b + c) < 0
    T[flip] = T[flip][:, [0, 2, 1]]
    return uniq, T


@dataclasses.dataclass
class Mesh:
    """MPAS-O mesh in the reference's storage convention (MPASOGrid members)."""
    nCells: int
    nVertices: int
    maxEdges: int
    nVertLevels: int
    cellCoord: np.ndarray          # [C,3] float64 (m)
    vertexCoord: np.ndarray        # [V,3] float64 (m)
    nEdgesOnCell: np.ndarray       # [C] uint64  (numberVertexOnCell_vec)
    verticesOnCell: np.ndarray     # [C*maxEdges] uint64, 1-based, 0 padded
    cellsOnCell: np.ndarray        # [C*maxEdges] uint64, 1-based, 0 = none
    cellsOnVertex: np.ndarray      # [V*3] uint64, 1-based, 0 = none
    refBottomDepth: np.ndarray     # [L] float64 (m, positive down)
    lat_cell: np.ndarray           # [C] rad
    lon_cell: np.ndarray           # [C] rad
    # edges (MPASOGrid edgesOnCell_vec / cellsOnEdge_vec / edgeCoord_vec): edge k of cell c lies
    # between its vertices k and k+1 and is shared with cellsOnCell[c, k]
    nEdges: int = 0
    edgesOnCell: np.ndarray = None   # [C*maxEdges] uint64, 1-based, 0 padded
    cellsOnEdge: np.ndarray = None   # [E*2] uint64, 1-based, 0 = culled (land) side
    edgeCoord: np.ndarray = None     # [E,3] float64 (m): the edge midpoint on the sphere

    @property
    def nVertLevelsP1(self) -> int:
        return self.nVertLevels + 1

    def nbytes(self) -> int:
        return sum(getattr(self, f).nbytes for f in
                   ("cellCoord", "vertexCoord", "nEdgesOnCell", "verticesOnCell",
                    "cellsOnCell", "cellsOnVertex"))


def _land_mask(lat, lon, kind: str):
    if kind == "none":
        return np.zeros(lat.shape, dtype=bool)
    # three "continents": spherical caps + a polar cap, ~10% of the sphere
    deg = np.degrees
    la, lo = deg(lat), deg(lon)

    def cap(lat0, lon0, rad):
        c0 = np.array([math.cos(math.radians(lat0)) * math.cos(math.radians(lon0)),
                       math.cos(math.radians(lat0)) * math.sin(math.radians(lon0)),
                       math.sin(math.radians(lat0))])
        xyz = np.stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)], 1)
        return xyz @ c0 > math.cos(math.radians(rad))

    m = cap(45.0, -100.0, 17.0) | cap(10.0, 20.0, 15.0) | cap(-25.0, 135.0, 12.0)
    m |= la < -80.0
    _ = lo
    return m


def _flip_edges(pts, T, n_flips: int, seed: int, max_deg: int):
    """Flip ``n_flips`` interior diagonals of the triangulation (vertex-disjoint, convex quads only):
    each turns two hexagonal Voronoi cells into pentagons and two into heptagons -- the 7-edge cells
    real MPAS meshes have and icosahedral duals lack (the RBF reconstruction's 7-point stencil,
    MPASOSolutionTBB.cpp:142, is only finite on them)."""
    if n_flips <= 0:
        return T
    T = T.copy()
    P = pts.shape[0]
    deg = np.bincount(T.reshape(-1), minlength=P)
    owner = {}
    for t in range(T.shape[0]):
        for i in range(3):
            owner[(int(T[t, i]), int(T[t, (i + 1) % 3]))] = t
    rng = np.random.default_rng(seed)
    used = np.zeros(P, dtype=bool)
    done = 0
    for t1 in rng.permutation(T.shape[0]):
        if done >= n_flips:
            break
        i = int(rng.integers(3))
        a, b, c = int(T[t1, i]), int(T[t1, (i + 1) % 3]), int(T[t1, (i + 2) % 3])
        t2 = owner.get((b, a))
        if t2 is None:
            continue
        d = [int(v) for v in T[t2] if v != a and v != b][0]
        if used[[a, b, c, d]].any() or deg[a] < 6 or deg[b] < 6 or deg[c] >= max_deg or deg[d] >= max_deg:
            continue
        ok = True
        for tri in ((a, d, c), (d, b, c)):  # both new triangles counter-clockwise from outside
            p0, p1, p2 = pts[tri[0]], pts[tri[1]], pts[tri[2]]
            if np.dot(np.cross(p1 - p0, p2 - p0), p0 + p1 + p2) <= 0.0:
                ok = False
        if not ok:
            continue
        T[t1] = (a, d, c)
        T[t2] = (d, b, c)
        deg[a] -= 1; deg[b] -= 1; deg[c] += 1; deg[d] += 1
        used[[a, b, c, d]] = True
        done += 1
    return T


def make_mesh(n: int, n_levels: int = 60, land: str = "continents", max_edges: int = 7,
              jitter: float = 0.05, seed: int = 7, radius: float = SPHERE_RADIUS,
              total_depth: float = 4000.0, flips: int = 0, edges: bool = True) -> Mesh:
    """``flips``: diagonal flips that give the mesh heptagons (and pentagons), see _flip_edges;
    ``edges``: also build the edge arrays (edgesOnCell, cellsOnEdge, edgeCoord)."""
    pts, T = geodesic_triangulation(n, jitter=jitter, seed=seed)
    T = _flip_edges(pts, T, flips, seed + 101, max_edges)
    P = pts.shape[0]
    a, b, c = pts[T[:, 0]], pts[T[:, 1]], pts[T[:, 2]]
    cc = np.cross(b - a, c - a)
    cc /= np.linalg.norm(cc, axis=1, keepdims=True)     # circumcentre direction
    # incidence (cell -> triangles), sorted CCW around the cell centre
    cell_of = T.reshape(-1)
    tri_of = np.repeat(np.arange(T.shape[0]), 3)
    ctr = pts[cell_of]
    ref = np.where(np.abs(ctr[:, 2:3]) < 0.9, np.array([[0.0, 0.0, 1.0]]), np.array([[1.0, 0.0, 0.0]]))
    e1 = np.cross(ref, ctr); e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
    e2 = np.cross(ctr, e1)
    cen = a + b + c
    cen /= np.linalg.norm(cen, axis=1, keepdims=True)
    d = cen[tri_of]             # fan order by triangle centroid (topological, robust)
    ang = np.arctan2(np.einsum("ij,ij->i", d, e2), np.einsum("ij,ij->i", d, e1))
    order = np.lexsort((ang, cell_of))
    cell_sorted = cell_of[order]
    tri_sorted = tri_of[order]
    deg = np.bincount(cell_of, minlength=P)
    if deg.max() > max_edges:
        raise ValueError(f"cell degree {deg.max()} exceeds maxEdges {max_edges}")
    start = np.concatenate([[0], np.cumsum(deg)[:-1]])
    kpos = np.arange(cell_sorted.size) - start[cell_sorted]
    voc = -np.ones((P, max_edges), dtype=np.int64)      # triangle (vertex) ids, 0-based
    voc[cell_sorted, kpos] = tri_sorted
    # neighbour k shares triangles k and k+1 (cyclic): the third corners of both
    coc = -np.ones((P, max_edges), dtype=np.int64)
    nxt = np.where(kpos + 1 < deg[cell_sorted], kpos + 1, 0)
    t0 = tri_sorted
    t1 = voc[cell_sorted, nxt]
    s0 = T[t0]; s1 = T[t1]
    # common corner other than the cell itself
    shared = -np.ones(t0.size, dtype=np.int64)
    for i in range(3):
        for j in range(3):
            hit = (s0[:, i] == s1[:, j]) & (s0[:, i] != cell_sorted)
            shared = np.where(hit & (shared < 0), s0[:, i], shared)
    coc[cell_sorted, kpos] = shared
    lat = np.arcsin(np.clip(pts[:, 2], -1, 1))
    lon = np.arctan2(pts[:, 1], pts[:, 0])

    # ---- cull land cells (MPAS culled-mesh convention) ----
    land_m = _land_mask(lat, lon, land)
    keep = ~land_m
    new_cell = -np.ones(P, dtype=np.int64)
    new_cell[keep] = np.arange(keep.sum())
    tri_keep = keep[T].any(axis=1)                      # vertex kept if it touches ocean
    new_vert = -np.ones(T.shape[0], dtype=np.int64)
    new_vert[tri_keep] = np.arange(tri_keep.sum())
    C = int(keep.sum()); V = int(tri_keep.sum())

    voc_k = voc[keep]
    coc_k = coc[keep]
    voc1 = np.where(voc_k >= 0, new_vert[np.maximum(voc_k, 0)] + 1, 0)
    coc_m = np.where(coc_k >= 0, new_cell[np.maximum(coc_k, 0)], -1)
    coc1 = np.where(coc_m >= 0, coc_m + 1, 0)
    cov = T[tri_keep]
    cov_m = new_cell[cov]
    cov1 = np.where(cov_m >= 0, cov_m + 1, 0)

    L = int(n_levels)
    # stretched reference layers: thin at the surface, thick at depth
    w = 1.0 + 4.0 * (np.arange(L) + 0.5) / L
    dz = total_depth * w / w.sum()
    refBottomDepth = np.cumsum(dz)

    edge_kw = {}
    if edges:
        # one edge per unordered neighbour pair (pre-cull ids); edge k of cell c joins its
        # vertices k and k+1 (the triangles it shares with neighbour k)
        kk = np.arange(max_edges)[None, :]
        valid = (kk < deg[:, None]) & (coc >= 0)
        ca = np.broadcast_to(np.arange(P)[:, None], coc.shape)
        lo = np.minimum(ca, coc); hi = np.maximum(ca, coc)
        key = np.where(valid, lo * np.int64(P) + hi, -1)
        ukeys, inv = np.unique(key[valid], return_inverse=True)
        eid = -np.ones(coc.shape, dtype=np.int64)
        eid[valid] = inv
        e_lo, e_hi = ukeys // P, ukeys % P
        e_keep = keep[e_lo] | keep[e_hi]  # MPAS culled meshes keep every edge of an ocean cell
        new_edge = -np.ones(ukeys.size, dtype=np.int64)
        new_edge[e_keep] = np.arange(e_keep.sum())
        # the edge's two vertices: (c, k) and (c, k+1) of any cell that has it
        cs, ks = np.nonzero(valid)
        k1 = np.where(ks + 1 < deg[cs], ks + 1, 0)
        ev = np.empty((ukeys.size, 2), dtype=np.int64)
        ev[eid[cs, ks], 0] = voc[cs, ks]
        ev[eid[cs, ks], 1] = voc[cs, k1]
        mid = cc[ev[:, 0]] + cc[ev[:, 1]]
        mid /= np.linalg.norm(mid, axis=1, keepdims=True)
        eoc = eid[keep]
        eoc1 = np.where(eoc >= 0, new_edge[np.maximum(eoc, 0)] + 1, 0)
        coe = np.stack([new_cell[e_lo[e_keep]], new_cell[e_hi[e_keep]]], axis=1)
        edge_kw = dict(nEdges=int(e_keep.sum()), edgesOnCell=eoc1.reshape(-1).astype(np.uint64),
                       cellsOnEdge=np.where(coe >= 0, coe + 1, 0).reshape(-1).astype(np.uint64),
                       edgeCoord=np.ascontiguousarray(mid[e_keep] * radius))

    return Mesh(
        **edge_kw,
        nCells=C, nVertices=V, maxEdges=max_edges, nVertLevels=L,
        cellCoord=np.ascontiguousarray(pts[keep] * radius),
        vertexCoord=np.ascontiguousarray(cc[tri_keep] * radius),
        nEdgesOnCell=deg[keep].astype(np.uint64),
        verticesOnCell=voc1.reshape(-1).astype(np.uint64),
        cellsOnCell=coc1.reshape(-1).astype(np.uint64),
        cellsOnVertex=cov1.reshape(-1).astype(np.uint64),
        refBottomDepth=refBottomDepth,
        lat_cell=lat[keep], lon_cell=lon[keep])


def frequency_for_cells(n_cells: int) -> int:
    return max(1, int(round(math.sqrt(max(n_cells - 2, 1) / 10.0))))


@dataclasses.dataclass
class Snapshot:
    """Raw per-cell MPAS-O history fields (MPASOSolution inputs)."""
    timestep: int
    layerThickness: np.ndarray     # [C*L]
    bottomDepth: np.ndarray        # [C]
    zonalVelocity: np.ndarray      # [C*L]
    meridionalVelocity: np.ndarray  # [C*L]
    vertVelocityTop: np.ndarray    # [C*(L+1)]
    attributes: dict               # name -> [C*L] (map order = sorted names)
    normalVelocity: np.ndarray = None  # [E*L] edge-normal velocity (make_snapshot(normal_velocity=True))


def make_snapshot(mesh: Mesh, timestep: int = 0, phase: float = 0.0, u0: float = 0.5,
                  u1: float = 0.25, w0: float = 1.0e-5, land_zero: bool = True,
                  inversions: float = 0.0, inversion_seed: int = 3, topography: str = "sigma",
                  normal_velocity: bool = False) -> Snapshot:
    """Solid-body flow + a travelling wave-3 perturbation, decaying with depth.

    ``normal_velocity``: also the MPAS edge-normal velocity [E*L] (``normalVelocity``, the input of
    the RBF reconstruction, MPASOSolutionTBB.cpp:131-245): the mean of the two cells' xyz velocity
    projected on the unit vector from cellsOnEdge[0] to cellsOnEdge[1]; 0 on boundary edges.

    ``phase`` (radians) shifts the perturbation eastward so consecutive daily
    snapshots form a time-varying (pathline) field.

    ``topography``: "sigma" stretches every layer by (bottom + ssh) / H, so each
    zTop column strictly decreases to the bottom; "zlevel" is MPAS-O's z-level
    grid with partial bottom cells: reference thicknesses down to the cell's
    bottom, the layer holding the bottom cut to it, zero thickness below
    (inactive levels, maxLevelCell), ssh added to the top layer -- zTop columns
    then end in flat runs and vertex columns mix cells of different depth.
    """
    C, L = mesh.nCells, mesh.nVertLevels
    lat, lon = mesh.lat_cell, mesh.lon_cell
    H = mesh.refBottomDepth[-1]
    # bottom depth: smooth bathymetry 2000..H
    bot = H - 0.5 * (H - 2000.0) * (1.0 + np.sin(2.0 * lat) * np.cos(3.0 * lon)) * 0.5
    bot = np.clip(bot, 1500.0, H)
    ref_dz = np.diff(np.concatenate([[0.0], mesh.refBottomDepth]))
    ssh = 0.5 * np.cos(lat) * np.sin(2.0 * lon + phase)
    if topography == "sigma":
        thick = ref_dz[None, :] * ((bot + ssh) / H)[:, None]
    elif topography == "zlevel":
        top = np.concatenate([[0.0], mesh.refBottomDepth[:-1]])
        thick = np.clip(bot[:, None] - top[None, :], 0.0, ref_dz[None, :])
        thick[:, 0] += ssh
    else:
        raise ValueError(f"unknown topography {topography!r}")
    if inversions > 0.0:
        # negative / zero layer thicknesses in a fraction of cells: the zTop
        # column is then non-monotone and the reference's fix-up (and the
        # engine's general bracket path) is exercised
        rng = np.random.default_rng(inversion_seed)
        sel = rng.random(C) < inversions
        lv = rng.integers(1, L - 1, size=C)
        rows = np.nonzero(sel)[0]
        thick[rows, lv[rows]] *= -0.5
        thick[rows, np.minimum(lv[rows] + 1, L - 1)] = 0.0
    # mid-layer depth (positive down) for the decay profile
    zmid = np.cumsum(thick, axis=1) - 0.5 * thick
    decay = np.exp(-zmid / 1500.0)
    cl = np.cos(lat)[:, None]
    u = (u0 * cl + u1 * np.cos(3.0 * lon - phase)[:, None] * np.sin(2.0 * lat)[:, None] * cl) * decay
    v = (u1 * np.sin(3.0 * lon - phase)[:, None] * cl * cl) * decay
    zi = np.concatenate([np.zeros((C, 1)), np.cumsum(thick, axis=1)], axis=1)   # interfaces
    wv = w0 * np.sin(2.0 * lat)[:, None] * np.sin(np.pi * zi / zi[:, -1:]) * np.cos(lon - phase)[:, None]
    temp = (2.0 + 25.0 * cl ** 2) * np.exp(-zmid / 800.0) + 1.0
    salt = 34.0 + 1.5 * np.sin(lat)[:, None] * np.exp(-zmid / 1000.0) + 0.1 * np.cos(2 * lon)[:, None]
    nvel = None
    if normal_velocity:
        if mesh.edgesOnCell is None:
            raise ValueError("normal_velocity needs a mesh built with edges=True")
        # ENU -> xyz at the cell centres (GeoConverter::convertENUVelocityToXYZ with w = 0)
        slon, clon, slat = np.sin(lon)[:, None], np.cos(lon)[:, None], np.sin(lat)[:, None]
        uxyz = np.stack([-slon * u - slat * clon * v, clon * u - slat * slon * v, cl * v], axis=-1)  # [C, L, 3]
        coe = mesh.cellsOnEdge.reshape(-1, 2).astype(np.int64) - 1
        inner = (coe >= 0).all(axis=1)
        a, b = coe[inner, 0], coe[inner, 1]
        nrm = mesh.cellCoord[b] - mesh.cellCoord[a]
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        nvel = np.zeros((mesh.nEdges, L))
        nvel[inner] = np.einsum("elk,ek->el", 0.5 * (uxyz[a] + uxyz[b]), nrm)
        nvel = np.ascontiguousarray(nvel.reshape(-1))
    return Snapshot(
        normalVelocity=nvel,
        timestep=timestep,
        layerThickness=np.ascontiguousarray(thick.reshape(-1)),
        bottomDepth=np.ascontiguousarray(bot),
        zonalVelocity=np.ascontiguousarray(u.reshape(-1)),
        meridionalVelocity=np.ascontiguousarray(v.reshape(-1)),
        vertVelocityTop=np.ascontiguousarray(wv.reshape(-1)),
        attributes={"salinity": np.ascontiguousarray(salt.reshape(-1)),
                    "temperature": np.ascontiguousarray(temp.reshape(-1))})


def latlon_to_xyz(lat_deg, lon_deg, r=SEED_RADIUS):
    """GeoConverter::convertDegreeToRadian + convertRadianLatLonToXYZ (GeoConverter.hpp:107-120, 176-186)."""
    lat = np.asarray(lat_deg, dtype=np.float64) * (math.pi / 180.0)
    lon = np.asarray(lon_deg, dtype=np.float64) * (math.pi / 180.0)
    ct, cp, st, sp = np.cos(lat), np.cos(lon), np.sin(lat), np.sin(lon)
    return np.stack([r * ct * cp, r * ct * sp, r * st], axis=-1)


def uniform_band_seeds(n: int, seed: int = 12345, max_abs_lat: float = 70.0, r: float = SEED_RADIUS):
    """Seeds uniform on the sphere band |lat| < max_abs_lat."""
    rng = np.random.default_rng(seed)
    zmax = math.sin(math.radians(max_abs_lat))
    z = rng.uniform(-zmax, zmax, n)
    lon = rng.uniform(-math.pi, math.pi, n)
    lat = np.degrees(np.arcsin(z))
    return latlon_to_xyz(lat, np.degrees(lon), r)


def gaussian_box_seeds(n: int, seed: int = 2024, mu=(25.0, -90.0), sigma=3.0,
                       lat_box=(18.0, 31.0), lon_box=(-98.0, -80.0), r: float = SEED_RADIUS):
    """Truncated Gaussian seeds (Gulf-of-Mexico box).

    Rejection per coordinate as MPASOVisualizer::GenerateGaussianSpherePoints
    (MPASOVisualizer.cpp:160-193), but with a fixed generator for reproducibility.
    """
    rng = np.random.default_rng(seed)
    out_lat = np.empty(n); out_lon = np.empty(n)
    filled = 0
    while filled < n:
        k = (n - filled) * 2 + 16
        la = rng.normal(mu[0], sigma, k); la = la[(la >= lat_box[0]) & (la <= lat_box[1])]
        lo = rng.normal(mu[1], sigma, k); lo = lo[(lo >= lon_box[0]) & (lo <= lon_box[1])]
        m = min(la.size, lo.size, n - filled)
        out_lat[filled:filled + m] = la[:m]; out_lon[filled:filled + m] = lo[:m]
        filled += m
    return latlon_to_xyz(out_lat, out_lon, r)


def lattice_seeds(n_lat: int, n_lon: int, lat_range, lon_range, depth: float = 0.0, r: float = SEED_RADIUS):
    """MPASOVisualizer::GenerateSamplePoint (MPASOVisualizer.cpp:120-149).

    Exclusive upper bounds: ``for (i = min; i < max; i += step)`` with
    ``step = (max-min)/(n-1)`` -- an 11x11 request yields 10x10 points.  The
    accumulation ``i += step`` is reproduced literally (floating-point drift
    included).
    """
    min_lat, max_lat = lat_range
    min_lon, max_lon = lon_range
    i_step = (max_lat - min_lat) / float(n_lat - 1)
    j_step = (max_lon - min_lon) / float(n_lon - 1)
    lats = []
    i = float(min_lat)
    while i < max_lat:
        lats.append(i)
        i += i_step
    lons = []
    j = float(min_lon)
    while j < max_lon:
        lons.append(j)
        j += j_step
    pts = []
    for la in lats:
        for lo in lons:
            pts.append((la, lo))
    if not pts:
        return np.zeros((0, 3))
    arr = np.array(pts)
    _ = depth
    return latlon_to_xyz(arr[:, 0], arr[:, 1], r)
