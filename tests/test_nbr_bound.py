"""CPU check of the neighbour-table stay test's error bound (dev::nbr_stay).

The device test keeps a particle in cell c without walking when, for every considered neighbour k,
g_k = fl32(h_k - 2 fl32(d_k . e)) > M_k = 2^-17 (h_k + |e|^2), with d_k = q_k - c rounded to float, e = p - c
formed in double and rounded to float, h_k = fl32(|d_k|^2).  The argument: |g_k - f_k| < 2^-20 (h_k + |e|^2) for
f_k = |p - q_k|^2 - |p - c|^2, so a passing test means the reference's double distances order c strictly
first.  Here numpy float32 arithmetic (one rounding per operation, as the kernel under -ffp-contract=off)
replays the test on points placed within 1e-6 m .. 1 km of real bisectors of the synthetic EC30to60-class and
oRRS-class meshes, at Earth radius, and every "stay" answer is checked against the distances computed the
reference's way (double, argmin with c last).  The stay ball it sets is checked the same way at 0.999 of its
radius.  The device's own test of the same function is tests/test_gpu_parity.py::test_neighbour_table_
shortcut_never_wrong."""
import numpy as np
import pytest


def _float_test(c, q, ok, p):
    """The kernel's arithmetic, vectorised: c [n,3], q [n,7,3] (neighbour centres), ok [n,7], p [n,3]."""
    f32 = np.float32
    d = (q - c[:, None, :]).astype(f32)                       # float offsets (cell_nbr_kernel)
    e = (p - c).astype(f32)                                   # (x - cx) in double, then rounded
    e2 = (e[:, 0] * e[:, 0] + e[:, 1] * e[:, 1]) + e[:, 2] * e[:, 2]
    h = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    dot = (d[..., 0] * e[:, None, 0] + d[..., 1] * e[:, None, 1]) + d[..., 2] * e[:, None, 2]
    g = h - f32(2.0) * dot
    M = f32(2.0 ** -17) * (h + e2[:, None])
    stay = np.all(~ok | (g > M), axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):  # (h = 0 in the masked slots)
        rk = np.where(ok, (g - M) * (f32(0.5) / np.sqrt(h)), np.inf).astype(np.float64)
    r = np.min(rk, axis=1) * (1.0 - 2.0 ** -16)
    return stay, r


def _walk_keeps(c, q, ok, p):
    """The reference's one-hop walk (MPASOVisualizerKernels.cpp:902-922, dev::walk): the first neighbour
    whose double distance is not above c's wins; c (listed last) only when every neighbour is farther."""
    dc = np.sqrt(np.sum((c - p) ** 2, axis=1))
    dn = np.sqrt(np.sum((q - p[:, None, :]) ** 2, axis=2))
    return np.all(~ok | (dn > dc[:, None]), axis=1)


@pytest.mark.parametrize("freq", [64, 158])
def test_float_bisector_test_never_keeps_a_cell_the_walk_leaves(freq):
    from mops_amd import synth
    mesh = synth.make_mesh(freq, n_levels=4)
    C = mesh.nCells
    me = mesh.maxEdges
    cc = np.asarray(mesh.cellCoord, dtype=np.float64).reshape(-1, 3)
    coc = np.asarray(mesh.cellsOnCell, dtype=np.int64).reshape(C, me) - 1
    ne = np.asarray(mesh.nEdgesOnCell, dtype=np.int64)
    rng = np.random.default_rng(freq)
    n = 60000
    cells = rng.integers(0, C, n)
    ids = np.full((n, 7), -1, dtype=np.int64)
    ids[:, :me] = coc[cells][:, :7]
    ok = (np.arange(7)[None, :] < ne[cells][:, None]) & (ids >= 0) & (ids < C)
    q = cc[np.where(ok, ids, cells[:, None])]
    c = cc[cells]
    # a point near the bisector with one (valid) neighbour, on either side, 1e-6 m .. 1 km from it
    k = np.array([rng.choice(np.flatnonzero(row)) for row in ok])
    qk = q[np.arange(n), k]
    dvec = qk - c
    nrm = dvec / np.linalg.norm(dvec, axis=1, keepdims=True)
    t = np.cross(nrm, c / np.linalg.norm(c, axis=1, keepdims=True))
    delta = np.sign(rng.uniform(-1, 1, n)) * 10.0 ** rng.uniform(-6, 3, n)
    tau = rng.uniform(-0.3, 0.3, n)[:, None] * np.linalg.norm(dvec, axis=1, keepdims=True)
    p = 0.5 * (c + qk) + delta[:, None] * nrm + tau * t
    p *= ((6371000.0 - rng.uniform(0.0, 5000.0, n)) / np.linalg.norm(p, axis=1))[:, None]
    stay, r = _float_test(c, q, ok, p)
    keeps = _walk_keeps(c, q, ok, p)
    assert not np.any(stay & ~keeps), "the float test kept a cell the walk leaves"
    assert stay[delta < -1.0].mean() > 0.5
    # the stay ball: 0.999 of its radius in random directions still keeps c
    sel = np.flatnonzero(stay & np.isfinite(r) & (r > 0.0))
    u = rng.normal(size=(len(sel), 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    p2 = p[sel] + 0.999 * r[sel, None] * u
    assert np.all(_walk_keeps(c[sel], q[sel], ok[sel], p2)), "a point inside the stay ball left the cell"
    print(f"freq {freq}: the float test answered for {stay.mean():.3f} of the points; the walk kept c for "
          f"{keeps.mean():.3f}")
