"""Parity at BASELINE.json's oRRS18to6-class sizes (configs 4 and 5).

The oRRS18to6-class synthetic mesh (frequency-608 icosahedral dual: 3.49M ocean
cells, 6.98M vertices, 80 levels) with the snapshots the configs-4/5 bench
streams through HBM: generated on the device (mops_amd/synth_device.py) and
derived in place (mops_field_create_device / mops_field_rebuild_device through
DeviceFieldRecycler, ~75 GB per field).  At this size

  * the level-pair records span 7.0M x 79 x 80 B = 44 GB per field, so their
    32-bit record indices (dev::pair_sums) and 64-bit byte addresses are used
    at scale;
  * the derived fields are exported from HBM (mops_field_export) and a random
    vertex subset is re-derived by the oracle from the same raw arrays
    (bitwise);
  * the trajectories run exactly as the bench runs them (PathlineChain with the
    field recycler; config 5 with its 3-day locality re-sorts inside a 30-day
    pair) and a random sample of lines (dead particles over-sampled) is
    re-run by the oracle on the exported fields: bit for bit.

Particles are independent, so a sampled particle's oracle line equals its line
in the full run whatever the other particles did.
"""
import types

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N_SNAP = 3  # config 4: two daily pairs (the second re-derives snapshot 0's buffers as snapshot 2)


@pytest.fixture(scope="module")
def orrs(gpu, engine_lib, oracle_lib):
    import torch
    from mops_amd import synth
    from mops_amd.engine import DeviceMesh
    from mops_amd.synth_device import DeviceSnapshotSource, device_field_factory
    mesh = synth.make_mesh(608, n_levels=80)
    dm = DeviceMesh.from_mesh(mesh)
    src = DeviceSnapshotSource(mesh, gpu)
    make = device_field_factory(dm, src)  # the same snapshots (phase 0.35 i) the recycler derives
    derived = []
    for i in range(N_SNAP):
        f = make(i, torch.cuda.current_stream(gpu).cuda_stream)
        zt, ve, w = f.export()
        derived.append(oracle_lib.Derived(zt, ve, w))
        f.close()
        del f
    torch.cuda.empty_cache()
    yield types.SimpleNamespace(mesh=mesh, dm=dm, src=src, derived=derived)
    torch.cuda.synchronize()


def _sample(n, dead_idx, k, k_dead, seed):
    rng = np.random.default_rng(seed)
    idx = rng.choice(n, k, replace=False)
    if dead_idx.size:
        idx = np.concatenate([idx, rng.choice(dead_idx, min(k_dead, dead_idx.size), replace=False)])
    return np.unique(idx)


def test_orrs_preprocessing_vertex_subset(orrs, oracle_lib):
    """Derived fields at oRRS size equal the oracle's preprocessing (MPASOSolutionTBB.cpp) on 4096
    random vertices, re-derived from the same raw device snapshot on the host."""
    import torch
    m = orrs.mesh
    V, L = m.nVertices, m.nVertLevels
    rng = np.random.default_rng(11)
    vids = np.sort(rng.choice(V, 4096, replace=False))
    cov = m.cellsOnVertex.reshape(V, 3)[vids].astype(np.int64)  # 1-based, 0 = missing (Q10)
    cells = np.unique(cov[cov > 0] - 1)
    sub_cov = np.where(cov > 0, np.searchsorted(cells, cov - 1) + 1, 0).astype(np.uint64)
    raw = orrs.src.make(timestep=0, phase=0.0)
    torch.cuda.synchronize()
    ci = torch.as_tensor(cells, device=raw["layerThickness"].device)
    take = lambda k: raw[k][ci].cpu().numpy().reshape(-1)
    snap = types.SimpleNamespace(layerThickness=take("layerThickness"), bottomDepth=take("bottomDepth"),
                                 zonalVelocity=take("zonalVelocity"), meridionalVelocity=take("meridionalVelocity"),
                                 vertVelocityTop=take("vertVelocityTop"), attributes={})
    sub = types.SimpleNamespace(nCells=len(cells), nVertices=len(vids), nVertLevels=L,
                                cellCoord=np.ascontiguousarray(m.cellCoord[cells]),
                                vertexCoord=np.ascontiguousarray(m.vertexCoord[vids]),
                                cellsOnVertex=np.ascontiguousarray(sub_cov.reshape(-1)))
    ref = oracle_lib.preprocess(sub, snap)
    d0 = orrs.derived[0]
    assert np.array_equal(d0.vertex_ztop.reshape(V, L)[vids].reshape(-1), ref.vertex_ztop)
    assert np.array_equal(d0.vertex_vel.reshape(V, L * 3)[vids].reshape(-1), ref.vertex_vel)
    assert np.array_equal(d0.vertex_w.reshape(V, L + 1)[vids].reshape(-1), ref.vertex_w)
    assert (cov == 0).any()  # boundary vertices (zero columns) are in the sample


def _chain(orrs, n_snap, gap):
    from mops_amd.chain import PathlineChain
    from mops_amd.synth_device import DeviceFieldRecycler
    rec = DeviceFieldRecycler(orrs.dm, orrs.src)
    return rec, PathlineChain(orrs.dm, rec, n_snap, gap_seconds=gap, own_fields=True, prefetch=False)


def _release(rec):
    import torch
    torch.cuda.synchronize()
    for f in rec.pool:
        f.close()
    rec.pool.clear()
    rec.raw = None
    torch.cuda.empty_cache()


def _check_lines(got, ref, idx):
    import torch
    ti = torch.as_tensor(idx, device=got["points"].device)
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        assert np.array_equal(got[k][ti].cpu().numpy(), ref[k]), k


def _check_shells(got, dead):
    """Every line of a particle alive through the whole chain is finite and stays on its shell.
    ``dead`` is the last pair's death steps: a particle that died in an earlier pair has zero records
    after its death (quirk Q1) and continues from there, so lines touching the origin are excluded."""
    import torch
    r = torch.linalg.norm(got["points"], dim=-1)
    live = torch.as_tensor(~dead, device=r.device) & (r.min(dim=1).values > 1e6)
    assert live.float().mean().item() > 0.9
    p = got["points"][live]
    assert torch.isfinite(p).all()
    rl = r[live]
    assert (rl - rl[:, :1]).abs().max().item() < 1e3


def test_config4_orrs_daily_pairs(orrs, oracle_lib):
    """BASELINE config 4 shape: 1e7 particles, depth 20 m, dt 120 s, daily pairs through the field
    recycler (2 pairs: snapshot 2 re-derived in snapshot 0's buffers), every line of a sample
    bit-exact against the oracle chain on the exported fields."""
    import bench
    from test_chain import oracle_chain
    seeds = bench.make_seeds(10_000_000, 0)
    rec, chain = _chain(orrs, N_SNAP, 86400)
    try:
        got = chain.run(seeds, depth=20.0, method=1, delta_t=120, record_t=3600)
        dead = got["death_step"].cpu().numpy() >= 0  # the last pair's deaths
        assert got["points"].shape == (len(seeds), 1 + 24 * (N_SNAP - 1), 3)
        idx = _sample(len(seeds), np.flatnonzero(dead), 256, 32, seed=41)
        ref = oracle_chain(oracle_lib, orrs.mesh, None, seeds[idx], 20.0, None, 86400, 120, 3600, euler=True,
                           derived=orrs.derived[:N_SNAP])
        _check_lines(got, ref, idx)
        _check_shells(got, dead)
    finally:
        del chain
        _release(rec)


def test_config5_orrs_monthly_pair(orrs, oracle_lib):
    """BASELINE config 5 shape, one monthly pair of the 365-day run on one GPU's share: 1.25e7
    Gaussian Gulf-of-Mexico particles, dt 60 s, 43 200 steps, recordT = 30 days (one record),
    launched as 3-day segments with a locality re-sort between them (PathlineChain's default)."""
    import bench
    from test_chain import oracle_chain
    seeds = bench.make_gaussian_seeds(12_500_000, 0)
    gap = 30 * 86400
    rec, chain = _chain(orrs, 2, gap)
    try:
        got = chain.run(seeds, depth=20.0, method=1, delta_t=60, record_t=gap)
        dead = got["death_step"].cpu().numpy() >= 0
        assert got["points"].shape == (len(seeds), 2, 3)
        idx = _sample(len(seeds), np.flatnonzero(dead), 192, 64, seed=53)
        ref = oracle_chain(oracle_lib, orrs.mesh, None, seeds[idx], 20.0, None, gap, 60, gap, euler=True,
                           derived=orrs.derived[:2])
        _check_lines(got, ref, idx)
        _check_shells(got, dead)
    finally:
        del chain
        _release(rec)
