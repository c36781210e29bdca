"""Parity at BASELINE.json's full sizes: the config-2 and
config-3 workloads on the EC30to60-class mesh (235 567 cells, 60 levels).

The oracle cannot run 1e6-1e7 particles for a day in seconds, so the full-size
checks are
  * a random sample of the SAME device run (particles are independent: every
    sampled line must equal the oracle's line for that seed, bit for bit,
    whatever the other particles did), dead particles over-sampled;
  * size-independent properties of the whole run: sharding the particle set
    (the multi-GPU partition, §8e) reproduces the unsharded records bit for bit,
    and every line of a live particle is finite and on its shell.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ec_case(gpu, engine_lib, oracle_lib):
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh
    mesh = synth.make_mesh(158, n_levels=60)
    s0 = synth.make_snapshot(mesh, timestep=0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    return mesh, dm, f0, f1, r0, r1


def _run_device(dm, f0, f1, cfg, seeds, depth):
    """Device-resident run (the bench path): returns seed cells, death steps and a
    lazily-indexable view of the finalized lines (seed order)."""
    import torch
    from mops_amd.engine import ParticleSet
    ps = ParticleSet(dm, seeds, depth, cfg)
    cells = ps.original(ps.cell).cpu().numpy()
    ps.advance(f0, f1, 0, cfg.n_steps)
    lines = ps.finalize(pathline=f1 is not None)
    death = ps.original(ps.death).cpu().numpy()
    torch.cuda.synchronize()
    return ps, cells, death, lines


def _sample(n, death, k=384, k_dead=64, seed=0):
    rng = np.random.default_rng(seed)
    dead = np.flatnonzero(death >= 0)
    idx = rng.choice(n, k, replace=False)
    if dead.size:
        idx = np.concatenate([idx, rng.choice(dead, min(k_dead, dead.size), replace=False)])
    return np.unique(idx)


def _check_sample(lines, death, idx, ref, pathline):
    import torch
    ti = torch.as_tensor(idx, device=lines["points"].device)
    pts = lines["points"][ti].cpu().numpy()
    vel = lines["velocity"][ti].cpu().numpy()
    assert np.array_equal(death[idx], ref["death"]), "death steps differ from the oracle"
    assert np.array_equal(pts, ref["points"]), "sampled lines differ from the oracle"
    assert np.array_equal(vel, ref["velocity"]), "sampled velocities differ from the oracle"
    assert np.array_equal(lines["lastPoint"][ti].cpu().numpy(), ref["lastPoint"])
    if pathline:
        assert np.array_equal(lines["temperature"][ti].cpu().numpy(), ref["temperature"])


def _check_shells(lines, death):
    """Every point of a particle that never died is finite and within 1 km of
    the sphere it started on (w*dt moves r by millimetres per step)."""
    import torch
    live = torch.as_tensor(death < 0, device=lines["points"].device)
    p = lines["points"][live]
    assert torch.isfinite(p).all()
    r = torch.linalg.norm(p, dim=-1)
    assert (r - r[:, :1]).abs().max().item() < 1e3


@pytest.mark.parametrize("method", [1, 0], ids=["euler", "rk4"])
def test_config1_lattice_every_line(ec_case, oracle_lib, method):
    """BASELINE config 1: the 100-seed GenerateSamplePoint lattice (11 x 11 request, exclusive upper
    bounds, lat [-40, 40], lon [-60, 60]) at "layer 10" (mid-depth of 0-based layer 10), dt 120 s,
    1-day streamline, through the host drop-in (mops_run_trajectories): every line bit-exact."""
    import bench
    from mops_amd import synth
    from mops_amd.engine import TrajectoryConfig, run_trajectories
    mesh, dm, f0, _, r0, _ = ec_case
    seeds = synth.lattice_seeds(11, 11, (-40.0, 40.0), (-60.0, 60.0))
    assert len(seeds) == 100
    depth = bench.layer_mid_depth(mesh, 10)
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=86400, recordT=3600, depth=depth, method=method)
    got = run_trajectories(dm, f0, None, cfg, seeds)
    ref = oracle_lib.run(mesh, r0, None, seeds, depth=depth, delta_t=120, duration=86400, record_t=3600,
                         euler=(method == 1))
    assert np.array_equal(got["cells"], ref["cells"])  # seed location = the oracle's exact 1-NN
    assert np.array_equal(got["death_step"], ref["death"])
    for k in ("points", "velocity", "lastPoint"):
        assert np.array_equal(got[k], ref[k]), k
    assert np.array_equal(got["final_depth"], ref["final_depth"])


def test_config2_full_size(ec_case, oracle_lib):
    """BASELINE config 2: 1e6 particles, depth 800 m, dt 120 s, 1-day Euler streamline."""
    import torch
    import bench
    from mops_amd.engine import TrajectoryConfig
    mesh, dm, f0, _, r0, _ = ec_case
    seeds = bench.make_seeds(1_000_000, 0)
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=86400, recordT=3600, depth=800.0, method=1)
    ps, cells, death, lines = _run_device(dm, f0, None, cfg, seeds, 800.0)
    idx = _sample(len(seeds), death)
    ref = oracle_lib.run(mesh, r0, None, seeds[idx], depth=800.0, delta_t=120, duration=86400, record_t=3600,
                         euler=True, cells=cells[idx])
    _check_sample(lines, death, idx, ref, pathline=False)
    _check_shells(lines, death)
    # the multi-GPU partition (contiguous shards, §8e) reproduces the unsharded run bit for bit
    half = len(seeds) // 2
    for lo, hi in ((0, half), (half, len(seeds))):
        _, _, d_s, l_s = _run_device(dm, f0, None, cfg, seeds[lo:hi], 800.0)
        assert np.array_equal(d_s, death[lo:hi])
        assert torch.equal(l_s["points"], lines["points"][lo:hi])
        assert torch.equal(l_s["velocity"], lines["velocity"][lo:hi])


def test_config2_full_size_rk4(ec_case, oracle_lib):
    """Config-2 shape with RK4 (Q1 cell-crossing deaths at full resolution)."""
    import bench
    from mops_amd.engine import TrajectoryConfig
    mesh, dm, f0, _, r0, _ = ec_case
    seeds = bench.make_seeds(1_000_000, 0)
    cfg = TrajectoryConfig(deltaT=120, simulationDuration=86400, recordT=3600, depth=800.0, method=0)
    _, cells, death, lines = _run_device(dm, f0, None, cfg, seeds, 800.0)
    assert (death >= 0).any()  # Q1 is exercised at this resolution
    idx = _sample(len(seeds), death, seed=1)
    ref = oracle_lib.run(mesh, r0, None, seeds[idx], depth=800.0, delta_t=120, duration=86400, record_t=3600,
                         euler=False, cells=cells[idx])
    _check_sample(lines, death, idx, ref, pathline=False)


def test_config3_full_size_pair(ec_case, oracle_lib):
    """BASELINE config 3, one daily pair: 1e7 particles at layer 10, dt 60 s, Euler pathline."""
    import bench
    from mops_amd.engine import TrajectoryConfig
    mesh, dm, f0, f1, r0, r1 = ec_case
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(10_000_000, 0)
    cfg = TrajectoryConfig(deltaT=60, simulationDuration=86400, recordT=3600, depth=depth, method=1)
    _, cells, death, lines = _run_device(dm, f0, f1, cfg, seeds, depth)
    idx = _sample(len(seeds), death, k=256, seed=2)
    ref = oracle_lib.run(mesh, r0, r1, seeds[idx], depth=depth, delta_t=60, duration=86400, record_t=3600,
                         euler=True, cells=cells[idx])
    _check_sample(lines, death, idx, ref, pathline=True)
    _check_shells(lines, death)


def test_config3_full_size_pair_rk4(ec_case, oracle_lib):
    """BASELINE config 3's pair with the north star's integrator (MOPSPathline.run's default, RK4): 1e7
    particles at layer 10, dt 60 s, one daily pair through the chain driver as the bench runs it -- dead-
    particle compaction between 6 launches, the cooperative-tile RK4 instantiation where waves share cells.
    Quirk Q1 kills a particle at its first cell crossing, so this also runs the compaction and the dead-
    particle records at full size; sampled lines (dead particles over-sampled) bit-exact against the oracle."""
    import torch
    import bench
    from mops_amd.chain import PathlineChain
    mesh, dm, f0, f1, r0, r1 = ec_case
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(10_000_000, 0)
    chain = PathlineChain(dm, lambda i, stream: (f0, f1)[i], 2, gap_seconds=86400, own_fields=False)
    got = chain.run(seeds, depth=depth, method=0, delta_t=60, record_t=3600, compact=True, compact_chunks=6)
    torch.cuda.synchronize()
    death = got["death_step"].cpu().numpy()
    assert 0.2 < (death >= 0).mean() < 0.95  # Q1 deaths throughout the day (and survivors)
    idx = _sample(len(seeds), death, k=256, k_dead=96, seed=4)
    cells = _locate(dm, seeds[idx])
    ref = oracle_lib.run(mesh, r0, r1, seeds[idx], depth=depth, delta_t=60, duration=86400, record_t=3600,
                         euler=False, cells=cells)
    _check_sample(got, death, idx, ref, pathline=True)
    _check_shells(got, death)


def _locate(dm, pts):
    import torch
    s = torch.as_tensor(np.ascontiguousarray(pts, dtype=np.float64), device="cuda")
    c = torch.empty((s.shape[0],), dtype=torch.int32, device="cuda")
    dm.locate(s.data_ptr(), c.data_ptr(), int(s.shape[0]))
    torch.cuda.synchronize()
    return c.cpu().numpy()


def test_config3_full_size_chain(ec_case, oracle_lib):
    """Config-3 shape through the pair-chaining driver (3 daily snapshots = 2 pairs, 1e6 particles):
    continuation seeds, the exact hinted seed location between pairs and the line concatenation at
    full mesh size.  Particles are independent across pairs too, so a sample's oracle chain (run on
    the sampled seeds alone) must reproduce the sampled lines bit for bit."""
    import torch
    import bench
    from test_chain import oracle_chain
    from mops_amd import synth
    from mops_amd.chain import PathlineChain
    mesh, dm, f0, f1, _, _ = ec_case
    snaps = [synth.make_snapshot(mesh, timestep=0), synth.make_snapshot(mesh, timestep=1, phase=0.35),
             synth.make_snapshot(mesh, timestep=2, phase=0.7)]
    from mops_amd.engine import DeviceField
    f2 = DeviceField.from_snapshot(dm, snaps[2])
    fields = [f0, f1, f2]
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(1_000_000, 0)
    chain = PathlineChain(dm, lambda i, stream: fields[i], 3, gap_seconds=86400, own_fields=False)
    got = chain.run(seeds, depth=depth, method=1, delta_t=60, record_t=3600)
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    idx = np.sort(rng.choice(len(seeds), 160, replace=False))
    ref = oracle_chain(oracle_lib, mesh, snaps, seeds[idx], depth, None, 86400, 60, 3600, euler=True)
    ti = torch.as_tensor(idx, device=got["points"].device)
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        assert np.array_equal(got[k][ti].cpu().numpy(), ref[k]), k
