"""CPU tests of the chain's pair schedule (calendar-month pairs, per-pair gaps from timestamps),
the bench's default workload, and the multi-GPU record collection (distributed.RecordGather)
over gloo with world size 2.

The month-pair and time-gap vectors are the reference's own functions' outputs
(tests/golden/month_pairs.json, made by tests/golden/make_month_pairs.py from
tutorial/pyMOPSAPI.py:1236-1295)."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden", "month_pairs.json")


def test_month_pairs_match_reference_vectors():
    from mops_amd import chain
    g = json.load(open(GOLD))
    for case in g["forward"]:
        assert [list(p) for p in chain.month_pairs_forward(*case["args"])] == case["pairs"], case["args"]
    for case in g["backward"]:
        assert [list(p) for p in chain.month_pairs_backward(*case["args"])] == case["pairs"], case["args"]


def test_time_gaps_match_reference_vectors():
    from mops_amd import chain
    g = json.load(open(GOLD))
    assert len(g["gaps"]) > 100
    for case in g["gaps"]:
        assert chain.time_gap_seconds(case["t1"], case["t2"]) == case["seconds"], (case["t1"], case["t2"])


def test_calendar_year_schedule():
    """Config 5's schedule: 12 calendar-month pairs from January = 365 days = 525 600 steps at dt 60."""
    from mops_amd import chain
    pairs = chain.month_pairs_forward(1, 1, 2, 1)
    ts = chain.month_timestamps(pairs)
    gaps = chain.pair_gaps(ts)
    assert len(pairs) == 12 and len(ts) == 13
    assert [g // 86400 for g in gaps] == [31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31]
    assert sum(gaps) // 60 == 525_600
    # backward: the same months in reverse, |gap| (pyMOPSAPI.py:1444 takes abs)
    back = chain.month_pairs_backward(2, 1, 1, 1)
    assert chain.pair_gaps(chain.month_timestamps(back)) == gaps[::-1]


def test_chain_accepts_per_pair_gaps_and_timestamps():
    from mops_amd.chain import PathlineChain
    ts = ["0001-01-01_00:00:00", "0001-02-01_00:00:00", "0001-03-01_00:00:00"]
    c = PathlineChain(None, None, 3, timestamps=ts)
    assert c.gaps == [31 * 86400, 28 * 86400]
    assert PathlineChain(None, None, 3, gap_seconds=[100, 200]).gaps == [100, 200]
    assert PathlineChain(None, None, 4, gap_seconds=600).gaps == [600] * 3
    with pytest.raises(ValueError):
        PathlineChain(None, None, 3, gap_seconds=[1, 2, 3])
    with pytest.raises(ValueError):
        PathlineChain(None, None, 3, timestamps=ts[:2])


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_bench_default_is_config3():
    """`python bench.py` (the driver's command) runs BASELINE config 3, the largest single-GPU config:
    1e7 particles, layer 10, dt 60 s, 7 daily pairs; config 5 runs the calendar year."""
    b = _bench()
    a = b.apply_config_defaults(b.parse(["--steps", "20", "--warmup", "5"]))
    assert (a.config, a.particles, a.dt, a.pairs, a.mode, a.method) == (3, 10_000_000, 60, 7, "pathline", "euler")
    assert (a.steps, a.warmup) == (20, 5)
    a = b.apply_config_defaults(b.parse([]))
    # the N > 1 collection the time model favours (a ring all-gather of config 3's records
    # is as long as the pair it overlaps; the gather to rank 0 moves one slab per link), and the caller-shaped
    # host delivery beside the device-resident value
    assert a.config == 3 and (a.steps, a.warmup) == (3, 1) and a.gather == "root" and a.deliver == "host"
    from mops_amd import chain
    assert chain.pair_gaps(b.chain_timestamps(3, 7)) == [86400] * 7
    a5 = b.apply_config_defaults(b.parse(["--config", "5"]))
    assert a5.pairs == 12 and a5.record == 86400 and (a5.steps, a5.warmup) == (1, 0)
    g5 = chain.pair_gaps(b.chain_timestamps(5, a5.pairs))
    assert sum(g // a5.dt for g in g5) == 525_600 and all(g % a5.record == 0 for g in g5)
    a2 = b.apply_config_defaults(b.parse(["--config", "2"]))
    assert (a2.particles, a2.dt, a2.mode) == (1_000_000, 120, "streamline")


class _Shard:
    """The parts of a ParticleSet that RecordGather reads: slot-ordered records, seeds and ids."""

    def __init__(self, records, seeds, ids, K):
        self.records, self.seeds, self.ids, self.K, self.n = records, seeds, ids, K, seeds.shape[0]

    def swap_records(self, slab):
        old, self.records = self.records, slab
        return old


def _gather_worker(rank, world, port, q, ring_records=1, mode="all"):
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from mops_amd import synth
    from mops_amd.distributed import RecordGather, max_shard, shard_bounds
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if mode == "rootfail":  # a backend without Gather: RecordGather falls back to the all-gather on every rank
        from mops_amd import distributed as D

        def _no_gather(*a, **k):
            raise RuntimeError("gather is not supported by this backend (test)")
        D.gather_flat = _no_gather
        mode = "root"
    try:
        mesh = synth.make_mesh(12, n_levels=8)
        snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.35 * t) for t in range(3)]
        d = [O.preprocess(mesh, s) for s in snaps]
        seeds = synth.uniform_band_seeds(91, seed=5)
        n_total = len(seeds)
        lo, hi = shard_bounds(n_total, rank, world)
        npad = max_shard(n_total, world)
        gaps = [14400, 7200]  # two chained pairs of different length: K = 4, then 2 records
        rng = np.random.default_rng(100 + rank)
        kmax = max(gaps) // 3600
        ok = True
        coll = None
        s_all = seeds
        for p, gap in enumerate(gaps):
            ref = O.run(mesh, d[p], d[p + 1], s_all, depth=200.0, delta_t=600, duration=gap, record_t=3600,
                        n_threads=1, finalize=False)
            K = gap // 3600
            # this rank's shard in a random slot order, as ParticleSet keeps it
            perm = rng.permutation(hi - lo)
            rec = torch.zeros((kmax, 6, npad), dtype=torch.float64)
            rec[:K, 0:3, : hi - lo] = torch.as_tensor(ref["rec_pos"][lo:hi][perm].transpose(1, 2, 0))
            rec[:K, 3:6, : hi - lo] = torch.as_tensor(ref["rec_vel"][lo:hi][perm].transpose(1, 2, 0))
            sd = torch.as_tensor(np.ascontiguousarray(s_all[lo:hi][perm]))
            ids = torch.as_tensor(perm.astype(np.int32))
            shard = _Shard(rec, sd, ids, K)
            if coll is None:
                coll = RecordGather(dist, shard, world, backend="gloo", mode=mode)
            coll.collect(shard)
            if coll.receives:
                got_rec, got_seeds = coll.unsharded(n_total)
                ok &= np.array_equal(got_rec[:, 0:3].numpy().transpose(2, 0, 1), ref["rec_pos"])
                ok &= np.array_equal(got_rec[:, 3:6].numpy().transpose(2, 0, 1), ref["rec_vel"])
                ok &= np.array_equal(got_seeds.numpy(), s_all)
            else:  # root mode: the senders hold no gathered records
                ok &= mode == "root" and rank > 0 and coll.gathered.numel() == 0
                try:
                    coll.unsharded(n_total)
                    ok = False
                except ValueError:
                    pass
            ok &= shard.records is not rec  # the particle set moved to the spare slab
            s_all = np.ascontiguousarray(ref["rec_pos"][:, K - 1])  # continuation points
        if mode == "root" and coll.mode == "root":  # (the ring / chunk checks below are the all-gather path's)
            pl = coll.plan()
            ok &= pl["mode"] == "root" and (pl["received_bytes_per_checkpoint"] > 0) == (rank == 0)
            q.put((rank, bool(ok)))
            return
        # bounded ring: the last checkpoint again, gathered in chunks of `ring_records` records through
        # on_chunk (max_bytes below one checkpoint's gathered slab: the multi-chunk path config 5 takes)
        chunks = []
        shard2 = _Shard(rec.clone(), sd, ids, K)
        ring = RecordGather(dist, shard2, world, backend="gloo", max_bytes=ring_records * world * 6 * npad * 8,
                            on_chunk=lambda g, k0, k1: chunks.append((k0, k1, g.clone())))
        ring.collect(shard2)
        want = [(k0, min(K, k0 + ring_records)) for k0 in range(0, K, ring_records)]
        ok &= ring.chunk == min(ring_records, kmax) and [c[:2] for c in chunks] == want
        pl = ring.plan()  # the memory plan bench.py prints for N > 1
        ok &= (pl["gathered_bytes_per_checkpoint"] == world * kmax * 6 * npad * 8 and pl["chunked"] == (ring.chunk < kmax)
               and pl["ring_bytes"] == world * (ring.chunk * 6 + 4) * npad * 8)
        whole = coll.gathered.view(-1)[: world * K * 6 * npad].view(world, K, 6, npad)
        ok &= torch.equal(torch.cat([c[2] for c in chunks], 1), whole)
        # the first pair's 4 records through the same ring: a ragged last chunk when ring_records = 3
        chunks.clear()
        rec0 = torch.zeros((kmax, 6, npad), dtype=torch.float64)
        rec0[:, :, : hi - lo] = torch.arange(kmax * 6 * (hi - lo), dtype=torch.float64).view(kmax, 6, -1) + 1e6 * rank
        shard3 = _Shard(rec0, sd, ids, kmax)
        ring.collect(shard3)
        want = [(k0, min(kmax, k0 + ring.chunk)) for k0 in range(0, kmax, ring.chunk)]
        ok &= [c[:2] for c in chunks] == want
        g = torch.cat([c[2] for c in chunks], 1)  # [world, kmax, 6, npad]
        for r in range(world):
            rlo, rhi = shard_bounds(n_total, r, world)
            exp = torch.arange(kmax * 6 * (rhi - rlo), dtype=torch.float64).view(kmax, 6, -1) + 1e6 * r
            ok &= torch.equal(g[r, :, :, : rhi - rlo], exp) and bool((g[r, :, :, rhi - rlo:] == 0).all())
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ring_records,mode", [(2, 1, "all"), (3, 3, "all"), (4, 1, "all"), (4, 3, "all"),
                                                     (8, 3, "all"), (8, 1, "root"), (3, 1, "root"),
                                                     (3, 1, "rootfail")])
def test_record_gather_gloo_chain_shaped(world, ring_records, mode):
    """Two chained pairs with different record counts: each rank's slot-ordered records, gathered by
    RecordGather and unsharded by the slot ids, equal the single-process (oracle) records bit for bit.
    91 particles: uneven, padded shards at 3 and 4 ranks (config 4's strong-scaling split of a
    non-divisible N); the bounded ring in chunks of 1 or 3 records (3: a ragged last chunk).  World 8 is the
    driver's scaling run's rank count; "root" is the Gather to rank 0 (bench.py's --gather root): rank 0's
    unsharded records equal the oracle's, the senders hold none."""
    import multiprocessing as mp
    import socket
    from oracle import oracle as O
    O.build()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q, ring_records, mode)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    res = dict(q.get(timeout=5) for _ in range(world))
    assert res == {r: True for r in range(world)}


def test_record_gather_collector_refuses_defer_lines():
    """PathlineChain.run(defer_lines=True) swaps the record slab before on_pair, so an on_pair that
    reads the pair's records is refused -- RecordGather.collect flags itself (reads_records), without the caller
    setting the attribute."""
    import torch
    from mops_amd.chain import PathlineChain
    from mops_amd.distributed import RecordGather
    shard = _Shard(torch.zeros((2, 6, 4), dtype=torch.float64), torch.zeros((4, 3), dtype=torch.float64),
                   torch.arange(4, dtype=torch.int32), 2)
    rg = RecordGather(None, shard, 1, backend="gloo")
    assert getattr(rg.collect, "reads_records", False)
    chain = PathlineChain(None, lambda i, stream: None, 2, gap_seconds=3600)
    with pytest.raises(ValueError, match="reads_records"):
        chain.run(np.zeros((4, 3)), depth=100.0, defer_lines=True, on_pair=rg.collect)


def test_gather_time_model():
    """DESIGN.md section 7's table: a ring all-gather moves (world-1) slabs through one xGMI link, a direct
    exchange (all-gather or Gather to rank 0) one slab per link in parallel; bench.py's config-3 slab at
    8 ranks: 11.5 GB per pair -> 0.53 s on a ring, 75 ms direct."""
    from mops_amd.distributed import XGMI_LINK_GBS, gather_seconds
    S = (24 * 6 + 4) * 10_000_000 * 8.0  # config 3: 24 records + seeds/ids per particle
    m = gather_seconds(S, 8)
    assert m["all_gather_ring"] == pytest.approx(7 * S / (XGMI_LINK_GBS * 1e9))
    assert m["all_gather_direct"] == m["root_direct"] == pytest.approx(S / (XGMI_LINK_GBS * 1e9))
    assert m["root_serial"] == m["all_gather_ring"]
    assert 0.5 < m["all_gather_ring"] < 0.6 and 0.07 < m["root_direct"] < 0.08
    assert gather_seconds(S, 1)["all_gather_ring"] == 0.0
