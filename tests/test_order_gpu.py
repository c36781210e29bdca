"""Particle locality ordering and record clearing on the device (no reference counterpart: the
reference never re-sorts its particles; these only have to be permutations that leave results
unchanged, which test_gpu_parity's compaction test checks end to end).

mops_order_particles[_live] sort by each particle's cell rank in the Morton order of the cell
centres (32-bit keys over particle_key_bits(C) bits), dead / cell-less particles last, stably;
mops_records_clear_dead zeroes the unsampled record slots of the dead tail after a compaction.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mesh_dev(gpu, engine_lib, small_case):
    from mops_amd.engine import DeviceMesh
    mesh = small_case[0]
    return mesh, DeviceMesh.from_mesh(mesh)


def _runs(seq):
    return 0 if len(seq) == 0 else 1 + int(np.count_nonzero(seq[1:] != seq[:-1]))


@pytest.mark.parametrize("n", [1, 63, 10007])
def test_order_particles_live_partition_and_stability(gpu, engine_lib, mesh_dev, n):
    import torch
    from mops_amd import _lib as L
    mesh, dm = mesh_dev
    Cn = mesh.nCells
    rng = np.random.default_rng(n)
    cells = rng.integers(0, Cn, n).astype(np.int32)
    cells[rng.random(n) < 0.05] = -1            # no cell: sorts with the dead
    cells[rng.random(n) < 0.02] = Cn            # out of range too
    death = np.where(rng.random(n) < 0.3, rng.integers(0, 500, n), -1).astype(np.int32)
    d_cells = torch.as_tensor(cells, device=gpu)
    d_death = torch.as_tensor(death, device=gpu)
    order = torch.empty(n, dtype=torch.int32, device=gpu)
    n_live = torch.full((1,), -7, dtype=torch.int32, device=gpu)
    nb = int(engine_lib.mops_order_scratch_bytes(n))
    assert nb > 0
    scratch = torch.empty(nb, dtype=torch.uint8, device=gpu)
    L.check(engine_lib.mops_order_particles_live(dm.handle, n, C.c_void_p(d_cells.data_ptr()),
                                                 C.c_void_p(d_death.data_ptr()), C.c_void_p(order.data_ptr()),
                                                 C.c_void_p(n_live.data_ptr()), C.c_void_p(scratch.data_ptr()),
                                                 nb, None), "mops_order_particles_live")
    # too small a scratch is refused
    assert engine_lib.mops_order_particles_live(dm.handle, n, C.c_void_p(d_cells.data_ptr()),
                                                C.c_void_p(d_death.data_ptr()), C.c_void_p(order.data_ptr()),
                                                None, C.c_void_p(scratch.data_ptr()), nb - 300, None) != 0
    torch.cuda.synchronize()
    o = order.cpu().numpy()
    live = (death < 0) & (cells >= 0) & (cells < Cn)
    nl = int(n_live.item())
    assert nl == int(live.sum())
    assert np.array_equal(np.sort(o), np.arange(n))             # a permutation
    assert live[o[:nl]].all() and not live[o[nl:]].any()        # live first
    assert np.all(np.diff(o[nl:]) > 0)                          # the rest keep their order (stable)
    c = cells[o[:nl]]
    assert _runs(c) == len(np.unique(c))                        # each cell's particles in one run
    for cc in np.unique(c)[:50]:                                # ... in slot order within it
        assert np.all(np.diff(o[:nl][c == cc]) > 0)
    # the same keys without deaths: mops_order_particles
    order2 = torch.empty(n, dtype=torch.int32, device=gpu)
    L.check(engine_lib.mops_order_particles(dm.handle, n, C.c_void_p(d_cells.data_ptr()),
                                            C.c_void_p(order2.data_ptr()), None), "mops_order_particles")
    torch.cuda.synchronize()
    o2 = order2.cpu().numpy()
    valid = (cells >= 0) & (cells < Cn)
    nv = int(valid.sum())
    assert valid[o2[:nv]].all() and np.all(np.diff(o2[nv:]) > 0)
    # live particles keep the relative order they have among all valid ones
    rank = np.empty(n, np.int64); rank[o2] = np.arange(n)
    assert np.all(np.diff(rank[o[:nl]]) > 0)


def test_order_is_spatially_local(gpu, engine_lib, mesh_dev):
    """Consecutive slots sit on nearby cells: the mean centre distance of neighbours in the
    sorted order is a small fraction of a random pairing's."""
    import torch
    from mops_amd import _lib as L
    mesh, dm = mesh_dev
    n = 20000
    cells = np.random.default_rng(3).integers(0, mesh.nCells, n).astype(np.int32)
    d_cells = torch.as_tensor(cells, device=gpu)
    order = torch.empty(n, dtype=torch.int32, device=gpu)
    L.check(engine_lib.mops_order_particles(dm.handle, n, C.c_void_p(d_cells.data_ptr()),
                                            C.c_void_p(order.data_ptr()), None), "mops_order_particles")
    torch.cuda.synchronize()
    xyz = np.asarray(mesh.cellCoord, dtype=np.float64)[cells[order.cpu().numpy()]]
    step = np.linalg.norm(np.diff(xyz, axis=0), axis=1).mean()
    rnd = np.linalg.norm(np.diff(np.asarray(mesh.cellCoord, dtype=np.float64)[cells], axis=0), axis=1).mean()
    assert step < 0.05 * rnd


@pytest.mark.parametrize("k_begin", [0, 2, 6])
def test_records_clear_dead(gpu, engine_lib, k_begin):
    import torch
    from mops_amd import _lib as L
    n, K, stride = 1000, 6, 1024
    rec = torch.rand((K, 6, stride), dtype=torch.float64, device=gpu) + 1.0
    before = rec.clone()
    n_live = torch.tensor([613], dtype=torch.int32, device=gpu)
    L.check(engine_lib.mops_records_clear_dead(n, C.c_void_p(n_live.data_ptr()), k_begin, K,
                                               C.c_void_p(rec.data_ptr()), stride, None), "mops_records_clear_dead")
    torch.cuda.synchronize()
    want = before.clone()
    want[k_begin:, :, 613:n] = 0.0
    assert torch.equal(rec, want)
    assert engine_lib.mops_records_clear_dead(n, C.c_void_p(n_live.data_ptr()), 0, K,
                                              C.c_void_p(rec.data_ptr()), n - 1, None) != 0  # stride < n
