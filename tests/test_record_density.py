"""The reference caller's record density at scale: MOPSPathline.run records every 6 minutes by default
(record_every_minutes=6, tutorial/pyMOPSAPI.py:1396,1476), K = 240 records per daily pair -- past the fused
assembly's 24-record tile, so the lines go through assemble_kernel + remove_nan_kernel.

* 1e6 particles, one daily pair on the EC30to60-class mesh, record_t 360 s, Euler and RK4, run the way the
  config-2 bench runs a call (two particle parts on their own streams, step chunks, RK4 with dead-particle
  compaction) with each part's lines assembled on its stream: sampled lines bit-exact against the oracle.
* The chain's writer hook (PathlineChain.run(on_lines=...)) hands the same lines over in slot chunks.
* 1e7 particles at K = 240 (a 115 GB record slab) through the writer hook without exhausting HBM.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ec_pair(gpu, engine_lib, oracle_lib):
    from mops_amd import synth
    from mops_amd.engine import DeviceField, DeviceMesh
    mesh = synth.make_mesh(158, n_levels=60)
    s0 = synth.make_snapshot(mesh, timestep=0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    dm = DeviceMesh.from_mesh(mesh)
    f0, f1 = DeviceField.from_snapshot(dm, s0), DeviceField.from_snapshot(dm, s1)
    r0, r1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    return mesh, dm, f0, f1, r0, r1


def _sample(n, death, k, k_dead, seed):
    rng = np.random.default_rng(seed)
    idx = rng.choice(n, k, replace=False)
    dead = np.flatnonzero(death >= 0)
    if dead.size:
        idx = np.concatenate([idx, rng.choice(dead, min(k_dead, dead.size), replace=False)])
    return np.unique(idx)


@pytest.mark.parametrize("method", [1, 0], ids=["euler", "rk4"])
def test_record_every_6_minutes_1e6(ec_pair, oracle_lib, method):
    import torch
    import bench
    from mops_amd.engine import ParticleSet, TrajectoryConfig
    mesh, dm, f0, f1, r0, r1 = ec_pair
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(1_000_000, 0)
    cfg = TrajectoryConfig(deltaT=60, simulationDuration=86400, recordT=360, depth=depth, method=method)
    assert cfg.n_records == 240
    ps = ParticleSet(dm, seeds, depth, cfg)
    cells = ps.original(ps.cell).cpu().numpy()
    streams = [torch.cuda.Stream() for _ in range(2)]
    ev = torch.cuda.Event(); ev.record()
    for st in streams:
        st.wait_event(ev)
    ps.advance_pipelined(f0, f1, 0, cfg.n_steps, streams, 6, compact=(method == 0))
    # each part's lines assembled on its own stream into the full outputs (the slot -> line map is what
    # the NaN cleanup must follow past 24 records)
    lines = ps.finalize(pathline=True, streams=streams)
    for st in streams:
        torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    death = ps.original(ps.death).cpu().numpy()
    if method == 0:
        assert (death >= 0).any()
    idx = _sample(len(seeds), death, 256, 64, seed=11 + method)
    ref = oracle_lib.run(mesh, r0, r1, seeds[idx], depth=depth, delta_t=60, duration=86400, record_t=360,
                         euler=(method == 1), cells=cells[idx])
    ti = torch.as_tensor(idx, device=lines["points"].device)
    assert np.array_equal(death[idx], ref["death"])
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        assert np.array_equal(lines[k][ti].cpu().numpy(), ref[k]), k
    assert lines["points"].shape[1] == 241


def test_writer_hook_hands_the_chain_lines_in_chunks(ec_pair):
    """PathlineChain.run(on_lines=...) at K = 240: every pair's lines in slot chunks with their particle ids
    -- scattered back, the same doubles as the concatenated lines of keep_lines (pair 1 without its first
    sample), and the continuation through mops_traj_last_points unchanged."""
    import torch
    import bench
    from mops_amd import synth
    from mops_amd.chain import PathlineChain
    from mops_amd.engine import DeviceField
    mesh, dm, f0, f1, _, _ = ec_pair
    f2 = DeviceField.from_snapshot(dm, synth.make_snapshot(mesh, timestep=2, phase=0.7))
    fields = [f0, f1, f2]
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(200_000, 1)
    n = len(seeds)
    chain = PathlineChain(dm, lambda i, stream: fields[i], 3, gap_seconds=86400, own_fields=False)
    kw = dict(depth=depth, method=1, delta_t=60, record_t=360)
    want = chain.run(seeds, **kw)
    got = {k: torch.full_like(v, float("nan")) for k, v in want.items()
           if k in ("points", "velocity", "temperature", "salinity")}
    calls = []

    def on_lines(p, lines, ids):
        col = slice(0, 241) if p == 0 else slice(241 + 240 * (p - 1), 241 + 240 * p)
        calls.append((p, int(ids.shape[0])))
        for k, v in lines.items():
            got[k][ids.long(), col] = v

    res = chain.run(seeds, keep_lines=False, on_lines=on_lines, lines_chunk=64_000, **kw)
    torch.cuda.synchronize()
    assert [c[0] for c in calls] == [0] * 4 + [1] * 4 and sum(c[1] for c in calls) == 2 * n
    for k in got:
        assert torch.equal(got[k], want[k]), k
    assert torch.equal(res["lastPoint"], want["lastPoint"])
    with pytest.raises(ValueError):
        chain.run(seeds, keep_lines=True, on_lines=on_lines, **kw)


@pytest.mark.parametrize("keep_all", [True, False])
def test_host_line_sink_delivers_the_device_lines(ec_pair, keep_all):
    """bench.py's host_delivery: chain.HostLineSink copies every pair's lines into pinned host
    buffers on a copy stream, overlapped with the next pair.  Scattered back by the row ids, the host lines
    are the same doubles as the device lines of keep_lines (pair 1 without its first sample).  K = 24 with an
    odd lines_chunk (the assembly's 16-B record reads at an odd slot offset) -- the chunks start at
    odd slots, where the record slab's base is not 16-B aligned."""
    import torch
    import bench
    from mops_amd import synth
    from mops_amd.chain import HostLineSink, PathlineChain
    from mops_amd.engine import DeviceField
    mesh, dm, f0, f1, _, _ = ec_pair
    f2 = DeviceField.from_snapshot(dm, synth.make_snapshot(mesh, timestep=2, phase=0.7))
    fields = [f0, f1, f2]
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(100_002, 2)  # an even record stride: the 16-B path is eligible
    n = len(seeds)
    chain = PathlineChain(dm, lambda i, stream: fields[i], 3, gap_seconds=86400, own_fields=False)
    kw = dict(depth=depth, method=1, delta_t=120, record_t=3600)
    want = chain.run(seeds, **kw)
    sink = HostLineSink(n, 24, "cuda", keep_all=keep_all)
    res = chain.run(seeds, keep_lines=False, on_lines=sink, lines_chunk=33_333, **kw)
    torch.cuda.synchronize()
    sink.synchronize()
    st = sink.d2h_stats()
    assert st["pairs"] == 2 and st["chunks"] == 2 * 4 and st["bytes"] > 2 * n * 24 * 64
    for p in (0, 1):
        h = sink.host(p)
        assert not h["points"].is_cuda and h["points"].is_pinned()
        ids = h["ids"].long()
        col = slice(0, 25) if p == 0 else slice(25, 49)
        for k in ("points", "velocity", "temperature", "salinity"):
            got = torch.empty_like(h[k])
            got[ids] = h[k]
            assert torch.equal(got, want[k][:, col].cpu()), (p, k)
    assert torch.equal(res["lastPoint"], want["lastPoint"])
    with pytest.raises(ValueError):  # sized for 100_002 lines: a bigger chain is refused, not written out of bounds
        sink(2, {k: torch.zeros((n + 1,) + tuple(v.shape[1:]), dtype=v.dtype, device="cuda")
                 for k, v in want.items() if k in ("points", "velocity", "temperature", "salinity")},
             torch.zeros(n + 1, dtype=torch.int32, device="cuda"))


def test_record_every_6_minutes_1e7_through_the_hook(ec_pair, oracle_lib):
    """1e7 particles, one daily pair at K = 240: the record slab alone is 1e7 x 240 x 48 B = 115 GB, and
    concatenated lines would add 154 GB; through the writer hook the lines live in 1e6-particle chunks.
    Sampled lines (taken from the chunks by particle id) bit-exact against the oracle."""
    import torch
    import bench
    from mops_amd.chain import PathlineChain
    mesh, dm, f0, f1, r0, r1 = ec_pair
    depth = bench.layer_mid_depth(mesh, 10)
    seeds = bench.make_seeds(10_000_000, 0)
    rng = np.random.default_rng(21)
    idx = np.sort(rng.choice(len(seeds), 192, replace=False))
    want = torch.as_tensor(idx, device="cuda")
    keep = torch.full((len(seeds),), -1, dtype=torch.int64, device="cuda")
    keep[want] = torch.arange(len(idx), device="cuda")
    pts = torch.empty((len(idx), 241, 3), dtype=torch.float64, device="cuda")
    vel = torch.empty_like(pts)
    seen = torch.zeros((), dtype=torch.int64, device="cuda")

    def on_lines(p, lines, ids):
        nonlocal seen
        j = keep[ids.long()]
        m = j >= 0
        pts[j[m]] = lines["points"][m]
        vel[j[m]] = lines["velocity"][m]
        seen = seen + ids.shape[0]

    chain = PathlineChain(dm, lambda i, stream: (f0, f1)[i], 2, gap_seconds=86400, own_fields=False)
    res = chain.run(seeds, depth=depth, method=1, delta_t=60, record_t=360, keep_lines=False, on_lines=on_lines,
                    lines_chunk=1_000_000)
    torch.cuda.synchronize()
    assert int(seen.item()) == len(seeds)
    from test_full_size import _locate
    cells = _locate(dm, seeds[idx])
    ref = oracle_lib.run(mesh, r0, r1, seeds[idx], depth=depth, delta_t=60, duration=86400, record_t=360,
                         euler=True, cells=cells)
    assert np.array_equal(res["death_step"].cpu().numpy()[idx], ref["death"])
    assert np.array_equal(pts.cpu().numpy(), ref["points"])
    assert np.array_equal(vel.cpu().numpy(), ref["velocity"])
    assert np.array_equal(res["lastPoint"].cpu().numpy()[idx], ref["lastPoint"])
