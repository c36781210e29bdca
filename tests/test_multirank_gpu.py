"""Two ranks on the one GPU of the test box (gloo, both on cuda:0): each rank runs a
real ``ParticleSet`` shard, whose records sit in slot (locality) order, and the
gathered slabs + slot ids must map back (``distributed.unshard_slots``) to the
single-process run bit for bit -- the exchange bench.py's N > 1 path performs over
RCCL, checked for usable output."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_SEEDS = 701
CFG = dict(deltaT=120, simulationDuration=43200, recordT=3600, depth=400.0, method=1)


def _case():
    from mops_amd import synth
    mesh = synth.make_mesh(16, n_levels=10)
    return mesh, synth.make_snapshot(mesh), synth.uniform_band_seeds(N_SEEDS, seed=23)


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mops_amd.distributed import max_shard, shard_bounds, unshard_slots
        from mops_amd.engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig
        torch.cuda.set_device(0)
        mesh, snap, seeds = _case()
        dm = DeviceMesh.from_mesh(mesh)
        f0 = DeviceField.from_snapshot(dm, snap)
        lo, hi = shard_bounds(len(seeds), rank, world)
        npad = max_shard(len(seeds), world)
        cfg = TrajectoryConfig(**CFG)
        ps = ParticleSet(dm, seeds[lo:hi], cfg.depth, cfg)
        ps.advance(f0, None, 0, cfg.n_steps)
        torch.cuda.synchronize()
        slab = torch.zeros((ps.K, 6, npad), dtype=torch.float64)
        slab[..., : hi - lo] = ps.records.cpu()
        ids = torch.full((npad,), -1, dtype=torch.int32)
        ids[: hi - lo] = ps.ids.cpu()
        assert not torch.equal(ids[: hi - lo], torch.arange(hi - lo, dtype=torch.int32)), "shard not permuted"
        outs = [torch.empty_like(slab) for _ in range(world)]
        outi = [torch.empty_like(ids) for _ in range(world)]
        dist.all_gather(outs, slab)
        dist.all_gather(outi, ids)
        if rank == 0:
            full = unshard_slots(torch.stack(outs), torch.stack(outi), len(seeds), world)
            q.put(full.numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_slot_order_gather_matches_single_run(gpu, engine_lib):
    import multiprocessing as mp
    import socket

    import torch
    from mops_amd.engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    mesh, snap, seeds = _case()
    dm = DeviceMesh.from_mesh(mesh)
    f0 = DeviceField.from_snapshot(dm, snap)
    cfg = TrajectoryConfig(**CFG)
    ps = ParticleSet(dm, seeds, cfg.depth, cfg)
    ps.advance(f0, None, 0, cfg.n_steps)
    ref = torch.empty_like(ps.records)
    ref[..., ps.ids.long()] = ps.records
    ref = ref.cpu().numpy()
    assert np.isfinite(ref).any() and np.abs(ref).max() > 0
    assert np.array_equal(got, ref)
