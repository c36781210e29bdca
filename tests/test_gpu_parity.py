"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Bar: BIT-EXACT.  Every comparison asserts np.array_equal (NaN patterns
included) on points, velocity, lastPoint, final depth and death steps: the
engine keeps the reference's operation order with FMA contraction off, and
device sqrt / division / sin / cos give the same doubles as the host's on
these inputs.  The north_star tolerance (endpoints within 1e-6 rad of the
reference) is strictly weaker; the angular error is still computed and
asserted so a failure message reports how far apart the results are.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_RAD = 1e-6


def ang_err(a, b):
    na = np.linalg.norm(a, axis=-1)
    nb = np.linalg.norm(b, axis=-1)
    both = (na > 0) & (nb > 0) & np.isfinite(na) & np.isfinite(nb)
    c = np.sum(a * b, -1) / np.where(both, na * nb, 1.0)
    ang = np.arccos(np.clip(c, -1.0, 1.0))
    return np.where(both, ang, 0.0), both


def assert_lines_match(got, ref, label):
    """Bit-exact match of one run against the oracle (see the module docstring)."""
    assert np.array_equal(got["death_step"], ref["death"]), f"{label}: death steps differ"
    for key in ("points", "lastPoint"):
        a, b = got[key], ref[key]
        # zero (never-written) slots and NaN padding must coincide exactly
        assert np.array_equal(np.linalg.norm(a, axis=-1) == 0, np.linalg.norm(b, axis=-1) == 0), f"{label} {key} zeros"
        assert np.array_equal(np.isfinite(a), np.isfinite(b)), f"{label} {key} NaN pattern"
        e, _ = ang_err(a, b)
        assert e.max() < TOL_RAD, f"{label} {key}: max angular error {e.max()} rad"
        assert np.array_equal(a, b, equal_nan=True), (
            f"{label} {key}: not bit-exact ({np.mean(np.all(a == b, axis=-1)):.6f} of points equal, "
            f"max angular error {e.max():.3e} rad)")
    assert np.array_equal(got["velocity"], ref["velocity"], equal_nan=True), f"{label}: velocity not bit-exact"
    assert np.array_equal(got["final_depth"], ref["final_depth"], equal_nan=True), f"{label}: depth not bit-exact"
    return float(np.mean(np.all(got["points"] == ref["points"], axis=-1)))


@pytest.fixture(scope="module")
def dev_small(gpu, engine_lib, small_case):
    from mops_amd.engine import DeviceField, DeviceMesh
    mesh, s0, s1 = small_case
    dm = DeviceMesh.from_mesh(mesh)
    return dm, DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)


@pytest.fixture(scope="module")
def ref_small(oracle_lib, small_case):
    mesh, s0, s1 = small_case
    return oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)


def test_device_math_matches_host(gpu):
    """sqrt / division must be correctly rounded on gfx950 (bit parity)."""
    import torch
    rng = np.random.default_rng(0)
    x = rng.uniform(1e-3, 1e14, 200000)
    t = torch.as_tensor(x, device=gpu)
    assert np.array_equal(torch.sqrt(t).cpu().numpy(), np.sqrt(x))
    y = rng.uniform(-1e7, 1e7, 200000)
    assert np.array_equal((torch.as_tensor(y, device=gpu) / t).cpu().numpy(), y / x)


def test_fast_math_helpers_match_library(gpu, engine_lib):
    """The kernel's exact sqrt and small-angle sincos (dev::xsqrt, dev::sincos_small) must
    give the device library's sqrt/sin/cos bit for bit; the library's correctly rounded
    sqrt must also equal the host's."""
    import ctypes
    import torch
    rng = np.random.default_rng(10)
    x = np.concatenate([10.0 ** rng.uniform(-320, 308, 400000), rng.uniform(0, 1e14, 200000),
                        np.array([0.0, -0.0, 5e-324, 2.0 ** -767, np.nextafter(2.0 ** -767, 0), np.inf, -1.0,
                                  np.nan, 1e-24, 4.0e13])])
    d = torch.as_tensor(x, device=gpu)
    out = torch.empty((len(x), 2), dtype=torch.float64, device=gpu)
    assert engine_lib.mops_selftest_math(len(x), ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(out.data_ptr()), 0,
                                         None) == 0
    o = out.cpu().numpy()
    assert np.array_equal(o[:, 0].view(np.int64), o[:, 1].view(np.int64)), "fast sqrt != sqrt()"
    fin = np.isfinite(x) & (x >= 0)
    assert np.array_equal(o[fin, 1], np.sqrt(x[fin]))
    th = np.concatenate([rng.uniform(-0.78, 0.78, 400000),
                         np.sign(rng.uniform(-1, 1, 400000)) * 10.0 ** rng.uniform(-14, np.log10(0.78), 400000),
                         rng.uniform(-1e-4, 1e-4, 1000000), np.array([0.0, -0.0, 0.7799999, -0.7799999, 1e-300])])
    d = torch.as_tensor(th, device=gpu)
    out = torch.empty((len(th), 4), dtype=torch.float64, device=gpu)
    assert engine_lib.mops_selftest_math(len(th), ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(out.data_ptr()), 1,
                                         None) == 0
    o = out.cpu().numpy()
    assert np.array_equal(o[:, 0].view(np.int64), o[:, 1].view(np.int64)), "fast sin != sin()"
    assert np.array_equal(o[:, 2].view(np.int64), o[:, 3].view(np.int64)), "fast cos != cos()"
    print(f"device sin == host sin: {np.mean(o[:, 1] == np.sin(th)):.6f}, cos: {np.mean(o[:, 3] == np.cos(th)):.6f}")
    # shared-reciprocal normalisation a / |a| (dev::xdiv_norm3) against three `/`, including
    # zero, signed-zero, subnormal, huge and non-finite components
    n = 600000
    sgn = np.sign(rng.uniform(-1, 1, (n, 3)))
    mags = np.concatenate([10.0 ** rng.uniform(-320, 308, (n // 3, 3)),            # any exponents
                           10.0 ** rng.uniform(-230, -200, (n // 6, 3)),           # near the 2^-700 bound
                           10.0 ** rng.uniform(88, 92, (n // 6, 3)),               # near the 2^300 bound
                           rng.uniform(0, 6.4e6, (n - n // 3 - 2 * (n // 6), 3))])  # trajectory-sized
    a = sgn * mags
    a[rng.uniform(size=(n, 3)) < 0.03] = 0.0
    a[rng.uniform(size=(n, 3)) < 0.01] = -0.0
    special = np.array([[0.0, 0.0, 1.0], [-0.0, 1.0, 1.0], [5e-324, 1.0, 0.0], [np.inf, 1.0, 1.0], [np.nan, 1.0, 1.0],
                        [2.0 ** -700, 1.0, 1.0], [np.nextafter(2.0 ** -700, 0), 1.0, 1.0], [2.0 ** 300, 0.0, 0.0],
                        [2.0 ** 300, 2.0 ** 300, 0.0], [1e-13, 0.0, 0.0], [1e-12, 1e-12, 1e-12]])
    a = np.concatenate([a, special])
    d = torch.as_tensor(a.reshape(-1), device=gpu)
    out = torch.empty((len(a), 6), dtype=torch.float64, device=gpu)
    assert engine_lib.mops_selftest_math(len(a), ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(out.data_ptr()), 2,
                                         None) == 0
    o = out.cpu().numpy()
    assert np.array_equal(o[:, :3].view(np.int64), o[:, 3:].view(np.int64)), "xdiv_norm3 != a / |a|"


def _walk_selftest(engine_lib, dm, pts, cells):
    import ctypes
    import torch
    d = torch.as_tensor(np.ascontiguousarray(pts, dtype=np.float64).reshape(-1), device="cuda")
    c = torch.as_tensor(np.ascontiguousarray(cells, dtype=np.int32), device="cuda")
    out = torch.empty((len(cells),), dtype=torch.int32, device="cuda")
    assert engine_lib.mops_selftest_walk(dm.handle, len(cells), ctypes.c_void_p(d.data_ptr()),
                                         ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(out.data_ptr()), None) == 0
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_neighbour_table_shortcut_never_wrong(gpu, engine_lib, medium_case):
    """dev::nbr_stay (the float bisector test that skips the one-hop walk) may only
    answer "c stays" where the walk keeps c: points placed on both sides of every cell's bisectors at
    1e-6 m .. 1 km, at radii through the water column, plus non-finite points; and every point inside the
    stay ball it sets (0.999 of its radius, random directions) keeps c under the walk too."""
    from mops_amd.engine import DeviceMesh
    mesh, _, _ = medium_case
    dm = DeviceMesh.from_mesh(mesh)
    rng = np.random.default_rng(77)
    cc = np.asarray(mesh.cellCoord, dtype=np.float64).reshape(-1, 3)
    coc = np.asarray(mesh.cellsOnCell, dtype=np.int64).reshape(mesh.nCells, -1)
    ne = np.asarray(mesh.nEdgesOnCell, dtype=np.int64)
    cells = rng.integers(0, mesh.nCells, 40000)
    slot = (rng.integers(0, 7, len(cells)) % ne[cells])
    nb = coc[cells, slot] - 1  # (1-based in the mesh arrays, 0 = none)
    keep = (nb >= 0) & (nb < mesh.nCells)
    cells, nb = cells[keep], nb[keep]
    c, q = cc[cells], cc[nb]
    d = q - c
    n = d / np.linalg.norm(d, axis=1, keepdims=True)
    t = np.cross(n, c / np.linalg.norm(c, axis=1, keepdims=True))
    delta = np.sign(rng.uniform(-1, 1, len(cells))) * 10.0 ** rng.uniform(-6, 3, len(cells))
    tau = rng.uniform(-0.3, 0.3, len(cells))[:, None] * np.linalg.norm(d, axis=1, keepdims=True)
    p = 0.5 * (c + q) + delta[:, None] * n + tau * t
    p *= ((6371000.0 - rng.uniform(0.0, 5000.0, len(cells))) / np.linalg.norm(p, axis=1))[:, None]
    # cell centres, interior points and non-finite points too
    p = np.concatenate([p, c[:500], c[:500] * 0.9999 + q[:500] * 0.0001,
                        np.array([[np.nan, 0, 0], [np.inf, 1, 1], [0, 0, 0]])])
    cells = np.concatenate([cells, cells[:500], cells[:500], np.array([0, 0, 0])])
    out = _walk_selftest(engine_lib, dm, p, cells)
    stay, walk_keeps = (out & 1) != 0, (out & 2) != 0
    assert not np.any(stay & ~walk_keeps), "the neighbour test kept a cell the walk leaves"
    inside = delta < -1.0  # clearly on c's side of this bisector
    print(f"nbr_stay answered for {stay.mean():.3f} of the points, {stay[:len(delta)][inside].mean():.3f} of those "
          f">1 m inside; the walk kept c for {walk_keeps.mean():.3f}")
    assert stay[:len(delta)][inside].mean() > 0.5  # (it answers for most interior points)
    # the stay ball: points at 0.999 of the radius in random directions keep c
    r = (out >> 8).astype(np.float64)
    sel = np.flatnonzero(stay & (r >= 1.0))[:20000]
    u = rng.normal(size=(len(sel), 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    p2 = p[sel] + 0.999 * r[sel, None] * u
    out2 = _walk_selftest(engine_lib, dm, p2, cells[sel])
    assert np.all((out2 & 2) != 0), "a point inside the stay ball left the cell"


def test_preprocessing_bitwise(dev_small, ref_small, small_case):
    mesh, s0, s1 = small_case
    _, f0, _ = dev_small
    r0, _ = ref_small
    zt, ve, w = f0.export()
    assert np.array_equal(zt, r0.vertex_ztop)
    assert np.array_equal(ve, r0.vertex_vel)
    assert np.array_equal(w, r0.vertex_w)


def test_locate_matches_bruteforce(gpu, dev_small, small_case, oracle_lib):
    import torch
    from mops_amd import synth
    mesh, _, _ = small_case
    dm, _, _ = dev_small
    pts = np.concatenate([synth.uniform_band_seeds(3000, seed=3, max_abs_lat=89.0),
                          synth.lattice_seeds(21, 21, (-60, 60), (-180, 180)),
                          mesh.cellCoord[:50] * 1.0,            # exact cell centres
                          np.zeros((3, 3)),                      # dead-particle continuation points
                          np.array([[1e3, -2e3, 5e2], [0.0, 0.0, 7e6]])])   # far off the sphere
    ref = oracle_lib.knn(mesh, pts)
    d = torch.as_tensor(pts, device=gpu)
    out = torch.empty(len(pts), dtype=torch.int32, device=gpu)
    dm.locate(d.data_ptr(), out.data_ptr(), len(pts))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    # hinted locate (chained pairs): the same answer for exact, neighbouring, random and invalid hints
    rng = np.random.default_rng(4)
    coc = mesh.cellsOnCell.astype(np.int64).reshape(mesh.nCells, -1) - 1
    nb = coc[np.clip(ref, 0, None), rng.integers(0, 5, len(ref))]
    for hint in (ref, nb, rng.integers(0, mesh.nCells, len(ref)), np.full(len(ref), -7)):
        hd = torch.as_tensor(np.ascontiguousarray(hint, dtype=np.int32), device=gpu)
        out.fill_(-99)
        dm.locate(d.data_ptr(), out.data_ptr(), len(pts), d_hint=hd.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("method", ["euler", "rk4"])
@pytest.mark.parametrize("direction", ["forward", "backward"])
def test_streamline_parity(dev_small, ref_small, small_case, oracle_lib, method, direction):
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, _ = dev_small
    r0, _ = ref_small
    seeds = np.concatenate([synth.lattice_seeds(11, 11, (-40.0, 40.0), (-60.0, 60.0)),
                            synth.uniform_band_seeds(400, seed=11)])
    depth = 800.0
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=86400, recordT=3600, depth=depth,
                           method=1 if method == "euler" else 0, direction=0 if direction == "forward" else 1)
    got = run_trajectories(dm, f0, None, cfg, seeds)
    ref = oracle_lib.run(mesh, r0, None, seeds, depth=depth, delta_t=120, duration=86400, record_t=3600,
                         euler=(method == "euler"), backward=(direction == "backward"), cells=got["cells"])
    exact = assert_lines_match(got, ref, f"streamline {method} {direction}")
    print(f"bit-exact points: {exact:.4f}")


@pytest.mark.parametrize("method", ["euler", "rk4"])
def test_pathline_backward_parity(dev_small, ref_small, small_case, oracle_lib, method):
    """PathLine with directionType backward (signed deltaT, Q7) through the alpha ramp and RK4 stage alphas."""
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    seeds = synth.uniform_band_seeds(400, seed=15)
    cfg = TrajectoryConfig(deltaT=300, simulationDuration=43200, recordT=3600, depth=450.0,
                           method=1 if method == "euler" else 0, direction=1)
    got = run_trajectories(dm, f0, f1, cfg, seeds)
    ref = oracle_lib.run(mesh, r0, r1, seeds, depth=450.0, delta_t=300, duration=43200, record_t=3600,
                         euler=(method == "euler"), backward=True, cells=got["cells"])
    assert_lines_match(got, ref, f"pathline backward {method}")
    assert np.array_equal(got["points"], ref["points"])


@pytest.mark.parametrize("method", ["euler", "rk4"])
def test_pathline_parity(dev_small, ref_small, small_case, oracle_lib, method):
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    seeds = synth.uniform_band_seeds(500, seed=5)
    rng = np.random.default_rng(9)
    depths = rng.uniform(5.0, 1500.0, len(seeds)).astype(np.float32)
    cfg = TrajectoryConfig(deltaT=60, simulationDuration=86400, recordT=3600, depth=0.0,
                           method=1 if method == "euler" else 0)
    got = run_trajectories(dm, f0, f1, cfg, seeds, depths=depths)
    ref = oracle_lib.run(mesh, r0, r1, seeds, depths=depths, delta_t=60, duration=86400, record_t=3600,
                         euler=(method == "euler"), cells=got["cells"])
    exact = assert_lines_match(got, ref, f"pathline {method}")
    assert np.array_equal(got["temperature"], ref["temperature"])  # Q9: velocity x
    assert np.array_equal(got["salinity"], ref["salinity"])        # Q9: velocity y
    print(f"bit-exact points: {exact:.4f}")


@pytest.mark.parametrize("method", ["euler", "rk4"])
@pytest.mark.parametrize("variant", ["forward", "backward", "zlevel"])
def test_pathline_cooperative_waves(gpu, engine_lib, dev_small, ref_small, small_case, oracle_lib, variant, method):
    """Pathline waves that share cells (config 3's density: ~40 particles per cell) take the
    cooperative path -- each group's polygon, edge normals and hinted-layer records loaded once into the
    wave's LDS tile and kept until a lane's cell or layer changes (traj_kernel, MOPS_COOP_PE / _PR); waves
    with more than MOPS_COOP_G groups switch to per-lane normals, and in RK4 (MOPS_RK4_HANDOFF) a wave
    leaves the hexagon-tile kernel at its first step outside a hexagon or the tile and finishes in the
    cooperative one.  Dense cells with one or two depth groups, seeds on land (dead at step 0), particles
    dying later, a partial last wave; forward, backward (dt < 0), and MPAS z-level columns (partial
    bottom cells: hint misses change the groups) -- bit-exact against the oracle."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    if variant == "zlevel":
        z0 = synth.make_snapshot(mesh, timestep=0, topography="zlevel")
        z1 = synth.make_snapshot(mesh, timestep=1, phase=0.35, topography="zlevel")
        f0, f1 = DeviceField.from_snapshot(dm, z0), DeviceField.from_snapshot(dm, z1)
        r0, r1 = oracle_lib.preprocess(mesh, z0), oracle_lib.preprocess(mesh, z1)
    rng = np.random.default_rng(41)
    cc = np.asarray(mesh.cellCoord, dtype=np.float64).reshape(-1, 3)
    cells = rng.choice(mesh.nCells, 14, replace=False)
    seeds, depths = [], []
    for j, c in enumerate(cells):
        k = 45 + j  # uneven counts: groups straddle wave boundaries
        u = cc[c] / np.linalg.norm(cc[c])
        jit = rng.normal(size=(k, 3)) * 2.0e4
        p = u + (jit - np.outer(jit @ u, u)) / 6.371e6
        seeds.append(p / np.linalg.norm(p, axis=1, keepdims=True) * 6.37101e6)
        d = np.full(k, 300.0) if j < 7 else np.where(np.arange(k) % 2 == 0, 300.0, 1100.0)
        if variant == "zlevel":  # around the local bottom of the shallowest columns (1500-4000 m)
            d = np.where(np.arange(k) % 3 == 0, 1450.0 + 10.0 * j, d)
        depths.append(d)
    land = synth.uniform_band_seeds(400, seed=3)
    seeds.append(land[:37]); depths.append(np.full(37, 500.0))
    seeds = np.concatenate(seeds); depths = np.concatenate(depths).astype(np.float32)
    back = variant == "backward"
    euler = method == "euler"
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=43200, recordT=3600, depth=0.0, method=1 if euler else 0,
                           direction=1 if back else 0)
    got = run_trajectories(dm, f0, f1, cfg, seeds, depths=depths)
    ref = oracle_lib.run(mesh, r0, r1, seeds, depths=depths, delta_t=120, duration=43200, record_t=3600,
                         euler=euler, backward=back, cells=got["cells"])
    assert len(seeds) % 64 != 0
    assert_lines_match(got, ref, f"pathline cooperative waves ({variant}, {method})")
    assert (ref["death"] >= 0).any() and (ref["death"] < 0).any()
    if euler:
        assert (ref["death"] < 0).sum() > len(seeds) // 2


def test_record_rules_odd_periods(dev_small, ref_small, small_case, oracle_lib):
    """recordT not a multiple of deltaT (streamline run_time % recordT rule)."""
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    seeds = synth.uniform_band_seeds(200, seed=21)
    for back, rr in ((None, None), (f1, r1)):
        cfg = TrajectoryConfig(deltaT=120, simulationDuration=7200, recordT=300, depth=100.0)
        got = run_trajectories(dm, f0, back, cfg, seeds)
        ref = oracle_lib.run(mesh, r0, rr, seeds, depth=100.0, delta_t=120, duration=7200, record_t=300,
                             cells=got["cells"])
        assert_lines_match(got, ref, "odd record period")


def test_segmented_advance_equals_single(gpu, dev_small, small_case):
    import torch
    from mops_amd import synth
    from mops_amd.engine import ParticleSet, TrajectoryConfig
    dm, f0, _ = dev_small
    seeds = synth.uniform_band_seeds(1000, seed=8)
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=86400, recordT=3600, depth=500.0, method=0)
    a = ParticleSet(dm, seeds, 500.0, cfg)
    a.advance(f0, None, 0, cfg.n_steps)
    b = ParticleSet(dm, seeds, 500.0, cfg)
    for s in range(0, cfg.n_steps, 37):
        b.advance(f0, None, s, min(s + 37, cfg.n_steps))
    torch.cuda.synchronize()
    assert torch.equal(a.records, b.records)
    assert torch.equal(a.x, b.x) and torch.equal(a.death, b.death) and torch.equal(a.depth, b.depth)


def test_pipelined_advance_equals_single(gpu, dev_small, small_case):
    """ParticleSet.advance_pipelined (particle parts on 3 streams x 5 step chunks, the bench's
    config-2 schedule) gives the single launch's records and state bit for bit."""
    import torch
    from mops_amd import synth
    from mops_amd.engine import ParticleSet, TrajectoryConfig
    dm, f0, f1 = dev_small
    seeds = synth.uniform_band_seeds(3001, seed=18)
    for back, method in ((None, 1), (f1, 0)):
        cfg = TrajectoryConfig(deltaT=120, simulationDuration=43200, recordT=3600, depth=350.0, method=method)
        a = ParticleSet(dm, seeds, 350.0, cfg)
        a.advance(f0, back, 0, cfg.n_steps)
        b = ParticleSet(dm, seeds, 350.0, cfg)
        streams = [torch.cuda.Stream() for _ in range(3)]
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        b.advance_pipelined(f0, back, 0, cfg.n_steps, streams, 5)
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        assert torch.equal(a.records, b.records)
        for k in ("x", "y", "z", "depth", "cell", "death"):
            assert torch.equal(getattr(a, k), getattr(b, k)), k


@pytest.mark.parametrize("back_on,method", [(False, 0), (True, 0), (False, 1)], ids=["sr", "pr", "se"])
def test_dead_particle_compaction_is_result_invariant(gpu, dev_small, small_case, oracle_lib, back_on, method):
    """Dead-particle compaction (advance_pipelined(compact=True): each part re-sorted with its dead
    particles last before every chunk, records already written permuted along) leaves every line,
    death step and final state bit-identical to one plain launch -- with RK4's Q1 deaths happening
    throughout the run -- and puts each part's dead particles after its live ones."""
    import torch
    from mops_amd import synth
    from mops_amd.engine import ParticleSet, TrajectoryConfig
    mesh, s0, s1 = small_case
    dm, f0, f1 = dev_small
    back = f1 if back_on else None
    seeds = synth.uniform_band_seeds(4099, seed=23)
    cfg = TrajectoryConfig(deltaT=300, simulationDuration=86400, recordT=3600, depth=250.0, method=method)
    a = ParticleSet(dm, seeds, 250.0, cfg)
    a.advance(f0, back, 0, cfg.n_steps)
    la = a.finalize(pathline=back_on)
    b = ParticleSet(dm, seeds, 250.0, cfg)
    b.records.fill_(float("nan"))  # records need no clearing (every slot is written, zeros at death)
    streams = [torch.cuda.Stream() for _ in range(2)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    b.advance_pipelined(f0, back, 0, cfg.n_steps, streams, 7, compact=True)
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    lb = b.finalize(pathline=back_on)
    torch.cuda.synchronize()
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        assert torch.equal(la[k], lb[k]), k
    for k in ("x", "y", "z", "depth", "cell", "death"):
        assert torch.equal(a.original(getattr(a, k)), b.original(getattr(b, k))), k
    death = b.original(b.death).cpu().numpy()
    if method == 0:
        assert (death >= 0).sum() > 50 and (death > 0).any()  # Q1 deaths during the run
    # a second run of the same set over the first run's records, its lines assembled per part on
    # the part streams (bench.py's overlapped finalize)
    c_seeds = torch.as_tensor(seeds, dtype=torch.float64, device=gpu)
    b.reseed(c_seeds, 250.0)
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    b.advance_pipelined(f0, back, 0, cfg.n_steps, streams, 5, compact=True)
    lc = b.finalize(pathline=back_on, streams=streams)
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        assert torch.equal(la[k], lc[k]), k
    # the oracle agrees on a sample (the compaction moved dead particles between waves)
    r0 = oracle_lib.preprocess(mesh, s0)
    r1 = oracle_lib.preprocess(mesh, s1) if back_on else None
    idx = np.unique(np.concatenate([np.arange(0, 4099, 37), np.flatnonzero(death >= 0)[:40]]))
    # seed cells: the oracle's own exact 1-NN (= mops_locate_cells, test_locate_matches_bruteforce)
    ref = oracle_lib.run(mesh, r0, r1, seeds[idx], depth=250.0, delta_t=300, duration=86400, record_t=3600,
                         euler=(method == 1))
    assert np.array_equal(lb["points"][torch.as_tensor(idx, device=gpu)].cpu().numpy(), ref["points"])
    assert np.array_equal(death[idx], ref["death"])


def test_medium_mesh_l60_parity(gpu, engine_lib, medium_case, oracle_lib):
    """EC30to60-like vertical grid (60 levels): exercises the streaming bracket."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh, TrajectoryConfig, run_trajectories
    mesh, s0, s1 = medium_case
    dm = DeviceMesh.from_mesh(mesh)
    f0 = DeviceField.from_snapshot(dm, s0)
    r0 = oracle_lib.preprocess(mesh, s0)
    zt, ve, w = f0.export()
    assert np.array_equal(zt, r0.vertex_ztop) and np.array_equal(ve, r0.vertex_vel)
    seeds = synth.uniform_band_seeds(2000, seed=12345)
    rng = np.random.default_rng(1)
    depths = rng.choice(np.array([0.0, 20.0, 800.0, 2500.0, 5000.0], dtype=np.float32), len(seeds))
    for method in (1, 0):
        cfg = TrajectoryConfig(deltaT=120, simulationDuration=43200, recordT=3600, depth=0.0, method=method)
        got = run_trajectories(dm, f0, None, cfg, seeds, depths=depths)
        ref = oracle_lib.run(mesh, r0, None, seeds, depths=depths, delta_t=120, duration=43200, record_t=3600,
                             euler=(method == 1), cells=got["cells"])
        assert_lines_match(got, ref, f"medium method={method}")


@pytest.mark.parametrize("method", ["euler", "rk4"])
def test_nonmonotone_columns(gpu, engine_lib, small_case, oracle_lib, method):
    """Inverted / zero-thickness layers: the reference's monotone fix-up fires
    and the engine must take its general (streaming) bracket path."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh, TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    s0 = synth.make_snapshot(mesh, timestep=0, inversions=0.4)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35, inversions=0.4, inversion_seed=4)
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    zt, _, _ = f0.export()
    assert np.array_equal(zt, r0.vertex_ztop)
    seeds = synth.uniform_band_seeds(600, seed=31)
    rng = np.random.default_rng(2)
    depths = rng.uniform(0.0, 3000.0, len(seeds)).astype(np.float32)
    for back, rb in ((None, None), (f1, r1)):
        cfg = TrajectoryConfig(deltaT=120, simulationDuration=43200, recordT=3600, depth=0.0,
                               method=1 if method == "euler" else 0)
        got = run_trajectories(dm, f0, back, cfg, seeds, depths=depths)
        ref = oracle_lib.run(mesh, r0, rb, seeds, depths=depths, delta_t=120, duration=43200, record_t=3600,
                             euler=(method == "euler"), cells=got["cells"])
        assert_lines_match(got, ref, f"nonmonotone {method} path={back is not None}")


def test_order_is_permutation_and_result_invariant(gpu, dev_small, small_case):
    import torch
    from mops_amd import synth
    from mops_amd.engine import ParticleSet, TrajectoryConfig
    dm, f0, f1 = dev_small
    seeds = synth.uniform_band_seeds(3000, seed=77)
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=21600, recordT=3600, depth=300.0, method=0)
    a = ParticleSet(dm, seeds, 300.0, cfg, use_order=True)
    b = ParticleSet(dm, seeds, 300.0, cfg, use_order=False)
    order = a.order.cpu().numpy()
    assert np.array_equal(np.sort(order), np.arange(len(seeds)))
    assert np.array_equal(np.sort(a.ids.cpu().numpy()), np.arange(len(seeds)))   # state physically permuted
    for ps in (a, b):
        ps.advance(f0, f1, 0, cfg.n_steps)
    la, lb = a.finalize(pathline=True), b.finalize(pathline=True)
    torch.cuda.synchronize()
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        assert torch.equal(la[k], lb[k]), k
    assert torch.equal(a.original(a.death), b.death) and torch.equal(a.original(a.x), b.x)
    # re-ordering mid-run permutes the records already written, results unchanged
    c = ParticleSet(dm, seeds, 300.0, cfg, use_order=True)
    c.advance(f0, f1, 0, 17)
    c.reorder()
    c.advance(f0, f1, 17, cfg.n_steps)
    lc = c.finalize(pathline=True)
    torch.cuda.synchronize()
    assert torch.equal(lc["points"], lb["points"]) and torch.equal(lc["velocity"], lb["velocity"])


@pytest.mark.parametrize("max_edges", [10, 16, 20])
def test_wide_stencil_instantiations(gpu, engine_lib, oracle_lib, max_edges):
    """maxEdges > 7 selects the MAXV 12 / 20 kernels (no register polygon
    cache, fewer waves); results must not depend on the padding width."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh, TrajectoryConfig, run_trajectories
    mesh = synth.make_mesh(16, n_levels=10, max_edges=max_edges)
    s0 = synth.make_snapshot(mesh, timestep=0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    seeds = synth.uniform_band_seeds(300, seed=41)
    for back, rb in ((None, None), (f1, r1)):
        for method in (1, 0):
            cfg = TrajectoryConfig(deltaT=300, simulationDuration=43200, recordT=3600, depth=250.0, method=method)
            got = run_trajectories(dm, f0, back, cfg, seeds)
            ref = oracle_lib.run(mesh, r0, rb, seeds, depth=250.0, delta_t=300, duration=43200, record_t=3600,
                                 euler=(method == 1), cells=got["cells"])
            assert_lines_match(got, ref, f"maxEdges={max_edges} path={back is not None} method={method}")
            assert np.array_equal(got["points"], ref["points"])


@pytest.mark.parametrize("levels", [2, 100, 101])
def test_level_count_bounds(gpu, engine_lib, oracle_lib, levels):
    """nVertLevels at the reference's bounds (MPASOVisualizerKernels.cpp:744-751:
    1 < L <= MAX_VERTICAL_LEVEL_NUM = 100): L = 2 (a single layer) and L = 100
    bit-exact against the oracle at depths through the whole column; L = 101 is
    refused per particle, so every line dies at step 0 as in the reference."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh, TrajectoryConfig, run_trajectories
    mesh = synth.make_mesh(16, n_levels=levels)
    s0 = synth.make_snapshot(mesh, timestep=0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    seeds = synth.uniform_band_seeds(200, seed=43)
    depths = np.random.default_rng(5).uniform(-50.0, 4500.0, len(seeds)).astype(np.float32)
    for back, rb in ((None, None), (f1, r1)):
        for method in (1, 0):
            cfg = TrajectoryConfig(deltaT=300, simulationDuration=21600, recordT=3600, depth=0.0, method=method)
            got = run_trajectories(dm, f0, back, cfg, seeds, depths=depths)
            ref = oracle_lib.run(mesh, r0, rb, seeds, depths=depths, delta_t=300, duration=21600, record_t=3600,
                                 euler=(method == 1), cells=got["cells"])
            label = f"L={levels} path={back is not None} method={method}"
            assert_lines_match(got, ref, label)
            assert np.array_equal(got["points"], ref["points"]), label
            if levels > 100:
                assert np.all(got["death_step"] == 0), label
            else:
                assert np.mean(got["death_step"] < 0) > 0.5, label


def test_edge_case_seeds(dev_small, ref_small, small_case, oracle_lib):
    """Edge cases the reference meets in practice, mixed into ordinary waves:
    seeds over culled land (nearest cell is coastal, IsInMesh fails: death at
    step 0), non-finite seeds (no cell, MPASOVisualizerKernels.cpp:744-753 guard),
    the origin (a chained dead particle's lastPoint, Q1), seeds exactly on cell
    centres and exactly on mesh vertices (equidistant from three centres: the
    argmin tie and the IsInMesh boundary), and seed depths above the surface,
    at 0 and below the bottom (Q5 clamp, bracket end cases)."""
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    land = synth.latlon_to_xyz(np.array([45.0, 47.0, 10.0, 12.0, -25.0, -85.0]),
                               np.array([-100.0, -98.0, 20.0, 22.0, 135.0, 10.0]))
    bad = np.array([[np.nan, 0.0, 0.0], [0.0, np.inf, 1.0], [0.0, 0.0, 0.0]])
    scale = synth.SEED_RADIUS / np.linalg.norm(mesh.cellCoord[0])
    centres = mesh.cellCoord[::97][:24] * scale
    verts = mesh.vertexCoord[::131][:24] * scale
    ocean = synth.uniform_band_seeds(64, seed=77)
    seeds = np.concatenate([ocean[:20], land, bad, centres, ocean[20:40], verts, ocean[40:]])
    rng = np.random.default_rng(3)
    depths = rng.uniform(10.0, 3000.0, len(seeds)).astype(np.float32)
    depths[::7] = -10.0
    depths[1::7] = 0.0
    depths[2::7] = 1.0e6
    for back, rb in ((None, None), (f1, r1)):
        for method in (1, 0):
            cfg = TrajectoryConfig(deltaT=120, simulationDuration=21600, recordT=1800, depth=0.0, method=method)
            got = run_trajectories(dm, f0, back, cfg, seeds, depths=depths)
            ref = oracle_lib.run(mesh, r0, rb, seeds, depths=depths, delta_t=120, duration=21600, record_t=1800,
                                 euler=(method == 1), cells=got["cells"])
            label = f"edge seeds path={back is not None} method={method}"
            assert_lines_match(got, ref, label)
            assert np.array_equal(got["points"], ref["points"], equal_nan=True), label
            n_ocean, n_land = 20, len(land)
            # land seeds die before they move; non-finite seeds have no cell
            assert np.all(got["death_step"][n_ocean:n_ocean + n_land] == 0), label
            assert np.all(got["cells"][n_ocean + n_land:n_ocean + n_land + 2] == -1), label
    # seed cells: on-centre seeds locate to that centre (as the oracle's exact 1-NN);
    # on-vertex seeds to one of the tied nearest centres
    n0 = 20 + len(land) + len(bad)
    assert np.array_equal(got["cells"][n0:n0 + len(centres)], oracle_lib.knn(mesh, centres))
    nv0 = n0 + len(centres) + 20
    for q, c in zip(verts, got["cells"][nv0:nv0 + len(verts)]):
        d2 = np.sum((mesh.cellCoord - q) ** 2, axis=1)
        assert c >= 0 and d2[c] <= d2.min() * (1.0 + 1e-12)


def test_empty_and_single_particle(dev_small, ref_small, small_case, oracle_lib):
    """N = 0 returns empty lines without a launch (MPASOVisualizerKernels.cpp:663-665);
    N = 1 is one partially filled wave."""
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=7200, recordT=600, depth=300.0)
    for back in (None, f1):
        got = run_trajectories(dm, f0, back, cfg, np.zeros((0, 3)))
        assert got["points"].shape == (0, cfg.n_records + 1, 3)
        assert got["death_step"].shape == (0,)
    seed = synth.uniform_band_seeds(1, seed=5)
    for back, rb in ((None, None), (f1, r1)):
        got = run_trajectories(dm, f0, back, cfg, seed)
        ref = oracle_lib.run(mesh, r0, rb, seed, depth=300.0, delta_t=120, duration=7200, record_t=600,
                             cells=got["cells"])
        assert_lines_match(got, ref, f"single particle path={back is not None}")
        assert np.array_equal(got["points"], ref["points"])


@pytest.mark.parametrize("method", ["euler", "rk4"])
def test_coastal_cells_boundary_vertices(dev_small, ref_small, small_case, oracle_lib, method):
    """Cells with a boundary vertex (a cellsOnVertex entry on culled land, quirk Q10:
    every derived value there is 0, so its zTop column is identically zero) take the
    hinted fast bracket when at least 5% of the Wachspress weight sits on decreasing
    columns, and the general streaming bracket otherwise (dev::fast_ok).  Seeds walk
    from each coastal cell's centre towards its boundary vertices, so both sides of
    the 5% threshold and the coastline walk are exercised."""
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, _, _ = small_case
    dm, f0, f1 = dev_small
    r0, r1 = ref_small
    zt = r0.vertex_ztop.reshape(mesh.nVertices, -1)
    zero_v = np.all(zt == 0.0, axis=1)
    voc = mesh.verticesOnCell.astype(np.int64).reshape(mesh.nCells, -1) - 1
    ne = mesh.nEdgesOnCell.astype(np.int64)
    seeds = []
    for c in range(mesh.nCells):
        vs = [v for v in voc[c, : ne[c]] if zero_v[v]]
        if not vs or len(seeds) > 600:
            continue
        cc = mesh.cellCoord[c]
        for v in vs[:2]:
            for t in (0.2, 0.55, 0.85, 0.95, 0.99, 0.999):
                q = cc + t * (mesh.vertexCoord[v] - cc)
                seeds.append(q / np.linalg.norm(q) * synth.SEED_RADIUS)
    seeds = np.array(seeds)
    assert len(seeds) > 100, "the small mesh should have coastal cells"
    rng = np.random.default_rng(6)
    depths = rng.uniform(5.0, 2500.0, len(seeds)).astype(np.float32)
    for back, rb in ((None, None), (f1, r1)):
        cfg = TrajectoryConfig(deltaT=120, simulationDuration=21600, recordT=1800, depth=0.0,
                               method=1 if method == "euler" else 0)
        got = run_trajectories(dm, f0, back, cfg, seeds, depths=depths)
        ref = oracle_lib.run(mesh, r0, rb, seeds, depths=depths, delta_t=120, duration=21600, record_t=1800,
                             euler=(method == "euler"), cells=got["cells"])
        assert_lines_match(got, ref, f"coastal {method} path={back is not None}")
        assert (got["death_step"] < 0).sum() > len(seeds) // 4, "most coastal particles should survive"


@pytest.mark.parametrize("method", ["euler", "rk4"])
def test_zlevel_topography_partial_bottom(gpu, engine_lib, oracle_lib, method):
    """MPAS-O z-level columns: partial bottom cells and zero-thickness inactive levels
    make zTop columns end in flat runs, so each cell's fast bracket is limited to its
    strictly decreasing prefix km (dev::fast_ok); particles near or below the local
    bottom walk below the prefix with the reference's fix-up chained level by level
    (dev::bracket_mono), or fall back to the whole-column scan.  Depths
    span the surface, mid-column, the bottom region and below the deepest bottom."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh, TrajectoryConfig, run_trajectories
    mesh = synth.make_mesh(32, n_levels=60)
    s0 = synth.make_snapshot(mesh, timestep=0, topography="zlevel")
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35, topography="zlevel")
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    zt, _, _ = f0.export()
    assert np.array_equal(zt, r0.vertex_ztop)
    z = r0.vertex_ztop.reshape(mesh.nVertices, -1)
    assert np.mean(np.any(np.diff(z, axis=1) >= -1e-6, axis=1)) > 0.5, "columns should end in flat runs"
    seeds = synth.uniform_band_seeds(1500, seed=61)
    rng = np.random.default_rng(8)
    depths = np.concatenate([rng.uniform(0.0, 5200.0, 1000),
                             rng.choice(np.array([0.0, 5.0, 1500.0, 2000.0, 3000.0, 3999.0, 4500.0]), 500)])
    depths = depths.astype(np.float32)
    for back, rb in ((None, None), (f1, r1)):
        cfg = TrajectoryConfig(deltaT=120, simulationDuration=21600, recordT=1800, depth=0.0,
                               method=1 if method == "euler" else 0)
        got = run_trajectories(dm, f0, back, cfg, seeds, depths=depths)
        ref = oracle_lib.run(mesh, r0, rb, seeds, depths=depths, delta_t=120, duration=21600, record_t=1800,
                             euler=(method == "euler"), cells=got["cells"])
        assert_lines_match(got, ref, f"zlevel {method} path={back is not None}")


def test_heptagon_cells_all_modes(gpu, engine_lib, oracle_lib):
    """maxEdges 7 with heptagons (diagonal flips): the MAXV 7 kernels keep the IsInMesh
    normals of polygon slots 0-4 in LDS and compute slots 5-6 per evaluation
    (MOPS_LDS_COMPACT / MOPS_NRM_SLOTS), so seeds are placed in and around the
    heptagon (and pentagon) cells; every mode bit-exact against the oracle."""
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh, TrajectoryConfig, run_trajectories
    mesh = synth.make_mesh(16, n_levels=10, flips=40)
    nv = mesh.nEdgesOnCell.astype(np.int64)
    odd = np.flatnonzero(nv != 6)
    assert (nv == 7).sum() >= 10, "the test mesh must have heptagons"
    rng = np.random.default_rng(5)
    c = mesh.cellCoord[np.repeat(odd, 4)]
    c = c + rng.normal(scale=2.0e4, size=c.shape)  # ~20 km around the odd cells' centres
    c *= (synth.SEED_RADIUS / np.linalg.norm(c, axis=1))[:, None]
    seeds = np.concatenate([c, synth.uniform_band_seeds(200, seed=43)])
    s0 = synth.make_snapshot(mesh, timestep=0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    for back, rb in ((None, None), (f1, r1)):
        for method in (1, 0):
            cfg = TrajectoryConfig(deltaT=300, simulationDuration=43200, recordT=3600, depth=250.0, method=method)
            got = run_trajectories(dm, f0, back, cfg, seeds)
            ref = oracle_lib.run(mesh, r0, rb, seeds, depth=250.0, delta_t=300, duration=43200, record_t=3600,
                                 euler=(method == 1), cells=got["cells"])
            assert_lines_match(got, ref, f"heptagons path={back is not None} method={method}")
            in_hept = np.isin(got["cells"], np.flatnonzero(nv == 7))
            assert in_hept.sum() >= 20
