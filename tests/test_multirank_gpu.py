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


# ---------------------------------------------------------------- RecordGather: bench.py's N > 1 default
RK4_CFG = dict(deltaT=300, simulationDuration=43200, recordT=3600, depth=350.0, method=0)
CHAIN_TS = ["0001-01-01_00:00:00", "0001-01-01_06:00:00", "0001-01-01_08:00:00"]


def _stream_case():
    from mops_amd import synth
    mesh = synth.make_mesh(16, n_levels=10)
    return mesh, synth.make_snapshot(mesh), synth.uniform_band_seeds(N_SEEDS, seed=31)


def _run_stream_shard(ps, f0, cfg):
    """bench.py's config-2 call shape: two particle parts on their own streams, step chunks, RK4
    dead-particle compaction between chunks, per-part line assembly."""
    import torch
    cur = torch.cuda.current_stream()
    parts = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in parts:
        st.wait_stream(cur)
    ps.advance_pipelined(f0, None, 0, cfg.n_steps, parts, 4, compact=True)
    out = ps.finalize(False, streams=parts)
    for st in parts:
        cur.wait_stream(st)
    return out


def _gather_worker_stream(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mops_amd.distributed import RecordGather, max_shard, shard_bounds
        from mops_amd.engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig
        torch.cuda.set_device(0)
        mesh, snap, seeds = _stream_case()
        dm = DeviceMesh.from_mesh(mesh)
        f0 = DeviceField.from_snapshot(dm, snap)
        lo, hi = shard_bounds(len(seeds), rank, world)
        cfg = TrajectoryConfig(**RK4_CFG)
        ps = ParticleSet(dm, seeds[lo:hi], cfg.depth, cfg, record_stride=max_shard(len(seeds), world))
        coll = RecordGather(dist, ps, world, backend="gloo")
        outs = []
        for _ in range(2):  # two calls: the second writes the spare slab while the first one's is gathered
            ps.reset(depth=cfg.depth)
            dm.locate(ps.seeds.data_ptr(), ps.cell.data_ptr(), ps.n)
            ps.reorder()
            _run_stream_shard(ps, f0, cfg)
            coll.collect(ps, torch.cuda.current_stream())
            coll.synchronize()
            torch.cuda.synchronize()
            lines = coll.lines(len(seeds), pathline=False)
            torch.cuda.synchronize()
            outs.append({k: v.cpu().numpy() for k, v in lines.items()})
        if rank == 0:
            q.put(outs)
    finally:
        dist.destroy_process_group()


def _gather_worker_chain(rank, world, port, q, mode="all"):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mops_amd import synth
        from mops_amd.chain import PathlineChain, snapshot_field_factory
        from mops_amd.distributed import RecordGather, max_shard, shard_bounds
        from mops_amd.engine import DeviceMesh
        torch.cuda.set_device(0)
        mesh, _, seeds = _stream_case()
        snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.35 * t) for t in range(len(CHAIN_TS))]
        dm = DeviceMesh.from_mesh(mesh)
        lo, hi = shard_bounds(len(seeds), rank, world)
        chain = PathlineChain(dm, snapshot_field_factory(dm, lambda i: snaps[i]), len(snaps), timestamps=CHAIN_TS)
        coll = [None]
        pair_lines = []

        def on_pair(p, last, ps):
            if coll[0] is None:
                coll[0] = RecordGather(dist, ps, world, backend="gloo", mode=mode)
            coll[0].collect(ps, torch.cuda.current_stream())
            coll[0].synchronize()
            torch.cuda.synchronize()
            if coll[0].receives:  # (root mode: rank 0 only)
                pair_lines.append({k: v.cpu().numpy() for k, v in coll[0].lines(len(seeds), pathline=True).items()})

        chain.run(seeds[lo:hi], depth=300.0, method=1, delta_t=600, record_t=3600, keep_lines=False, on_pair=on_pair,
                  record_stride=max_shard(len(seeds), world))
        torch.cuda.synchronize()
        if rank == 0:
            q.put(pair_lines)
    finally:
        dist.destroy_process_group()


def _spawn(target, world=2, *extra):
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    return got


def test_two_rank_record_gather_rk4_compaction_matches_single_run(gpu, engine_lib):
    """bench.py config 2 at N > 1: RK4 with dead-particle compaction between step chunks
    permutes each rank's slots; the records, seeds and slot ids RecordGather takes after the call are
    in one consistent order, and the lines rebuilt from the gather equal the single-process lines bit
    for bit -- in two consecutive calls (the second writes the spare slab)."""
    from mops_amd.engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig
    got = _spawn(_gather_worker_stream)
    mesh, snap, seeds = _stream_case()
    dm = DeviceMesh.from_mesh(mesh)
    f0 = DeviceField.from_snapshot(dm, snap)
    cfg = TrajectoryConfig(**RK4_CFG)
    ps = ParticleSet(dm, seeds, cfg.depth, cfg)
    ps.advance(f0, None, 0, cfg.n_steps)
    ref = {k: v.cpu().numpy() for k, v in ps.finalize(False).items()}
    assert (ps.death >= 0).any(), "the case should kill particles (Q1) so that compaction permutes slots"
    for call in got:
        for k in ("points", "velocity", "lastPoint"):
            assert np.array_equal(call[k], ref[k]), k


@pytest.mark.parametrize("mode", ["all", "root"])
def test_two_rank_record_gather_chain_matches_single_run(gpu, engine_lib, mode):
    """bench.py configs 3-5 at N > 1: every pair's record slab gathered (pairs of 6 h and 2 h from the
    snapshots' timestamps), all-gathered or (bench.py's default, --gather root) gathered to rank 0; the
    gathered lines, concatenated as MOPSPathline.run does, equal the single-process chain's lines bit for bit."""
    from mops_amd import synth
    from mops_amd.chain import PathlineChain, snapshot_field_factory
    from mops_amd.engine import DeviceMesh
    got = _spawn(_gather_worker_chain, 2, mode)
    mesh, _, seeds = _stream_case()
    snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.35 * t) for t in range(len(CHAIN_TS))]
    dm = DeviceMesh.from_mesh(mesh)
    chain = PathlineChain(dm, snapshot_field_factory(dm, lambda i: snaps[i]), len(snaps), timestamps=CHAIN_TS)
    ref = chain.run(seeds, depth=300.0, method=1, delta_t=600, record_t=3600)
    assert len(got) == 2 and got[0]["points"].shape[1] == 7 and got[1]["points"].shape[1] == 3
    pts = np.concatenate([got[0]["points"], got[1]["points"][:, 1:]], 1)
    vel = np.concatenate([got[0]["velocity"], got[1]["velocity"][:, 1:]], 1)
    assert np.array_equal(pts, ref["points"].cpu().numpy())
    assert np.array_equal(vel, ref["velocity"].cpu().numpy())
    assert np.array_equal(got[1]["lastPoint"], ref["lastPoint"].cpu().numpy())
