"""CPU-side tests: synthetic meshes, the C ABI library surface (no GPU
compute), host logic, and the multi-rank sharding with gloo."""
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- meshes
@pytest.mark.parametrize("land", ["none", "continents"])
def test_mesh_is_valid_mpas_layout(land):
    from mops_amd import synth
    m = synth.make_mesh(12, n_levels=5, land=land)
    C, mE = m.nCells, m.maxEdges
    voc = m.verticesOnCell.reshape(C, mE).astype(np.int64) - 1
    coc = m.cellsOnCell.reshape(C, mE).astype(np.int64) - 1
    ne = m.nEdgesOnCell.astype(int)
    assert m.nVertices == m.cellsOnVertex.size // 3
    for c in range(C):
        p = m.cellCoord[c]
        for k in range(ne[c]):
            a, b = m.vertexCoord[voc[c, k]], m.vertexCoord[voc[c, (k + 1) % ne[c]]]
            assert np.dot(np.cross(a, b), p) > 0           # CCW, centre inside (IsInMesh)
            d = coc[c, k]
            if d >= 0:
                assert c in coc[d, : ne[d]]                # symmetric neighbours
        assert np.all(voc[c, ne[c]:] == -1)                # zero padding
    if land == "none":
        assert C == 10 * 12 ** 2 + 2 and np.all(coc[np.arange(mE)[None, :] < ne[:, None]] >= 0)
    else:
        assert (m.cellsOnVertex == 0).any()                # culled coast


def test_norm_threshold():
    """The engine tests `x*x+y*y+z*z < 0x1.357c299a88ea7p-80` in place of the
    reference's `length(v) < 1e-12` (kNormTiny2, mops_engine.hip): the constant
    is the smallest double whose correctly rounded sqrt is >= 1e-12."""
    import math
    import struct
    t = float.fromhex("0x1.357c299a88ea7p-80")
    below = struct.unpack("<d", struct.pack("<q", struct.unpack("<q", struct.pack("<d", t))[0] - 1))[0]
    assert math.sqrt(t) >= 1e-12 and math.sqrt(below) < 1e-12
    assert t == 1e-24
    rng = np.random.default_rng(0)
    s = np.concatenate([rng.uniform(0, 4e-24, 20000), [0.0, t, below, np.inf, np.nan]])
    assert np.array_equal(np.sqrt(s) < 1e-12, s < t)


def test_frequency_for_cells():
    from mops_amd import synth
    assert synth.frequency_for_cells(236000) in (153, 154)


# ---------------------------------------------------------------- C ABI
def _header_functions():
    src = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("mops_traj.h", "mops_io.h", "mops_netcdf.h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mops_[a-z_0-9]+)\s*\(", src)))


def test_abi_exports_every_header_symbol(engine_lib):
    from mops_amd import _lib
    names = _header_functions()
    assert set(names) == set(_lib.EXPORTED)
    for n in names:
        assert hasattr(engine_lib, n), n


def test_abi_host_only_calls(engine_lib):
    import ctypes as C
    from mops_amd import _lib
    assert engine_lib.mops_abi_version() == 4
    cfg = _lib.TrajCfg(120, 86400, 3600, 0, 1)
    assert engine_lib.mops_traj_num_records(C.byref(cfg)) == 24
    assert engine_lib.mops_traj_num_steps(C.byref(cfg)) == 720
    # invalid settings are rejected before any device work (reference: Error() + {})
    bad = _lib.TrajCfg(0, 86400, 3600, 0, 1)
    p = _lib.Particles(0, None, None, None, None, None, None, None)
    st = engine_lib.mops_traj_advance(None, None, None, C.byref(bad), C.byref(p), 0, 1, None, 0, None)
    assert st == _lib.MOPS_ERR_INVALID
    assert b"invalid" in engine_lib.mops_last_error()
    h = C.c_void_p()
    desc = _lib.MeshDesc(0, 0, 7, 60, None, None, None, None, None, None)
    assert engine_lib.mops_mesh_create(C.byref(desc), None, C.byref(h)) == _lib.MOPS_ERR_INVALID
    desc = _lib.MeshDesc(10, 10, 21, 60, None, None, None, None, None, None)
    assert engine_lib.mops_mesh_create(C.byref(desc), None, C.byref(h)) == _lib.MOPS_ERR_UNSUPPORTED


def test_library_missing_fails_loudly(tmp_path):
    from mops_amd import _lib
    with pytest.raises(_lib.MopsError):
        saved = _lib._lib
        try:
            _lib._lib = None
            _lib.load(str(tmp_path / "nope.so"))
        finally:
            _lib._lib = saved


def test_oracle_not_imported_by_product():
    """The product package never references the oracle (test infrastructure)."""
    pkg = os.path.join(ROOT, "mops_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
                assert "mops_oracle" not in txt and "orc_" not in txt, f


# ---------------------------------------------------------------- host logic
def test_shard_bounds_cover_exactly():
    from mops_amd.distributed import max_shard, shard_bounds
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in spans) == max_shard(n, w) or n == 0


def test_unshard_slots_inverts_any_slot_order():
    """Property: whatever locality permutation each rank applied to its shard, gathering
    the slot-ordered slabs (padded to the largest shard) with the ranks' slot ids and
    unsharding gives the global particle order back; an id outside its shard is rejected."""
    from hypothesis import given, settings, strategies as st
    from mops_amd.distributed import max_shard, shard_bounds, unshard_slots

    @settings(max_examples=60, deadline=None)
    @given(n=st.integers(0, 300), world=st.integers(1, 9), seed=st.integers(0, 2**31 - 1))
    def prop(n, world, seed):
        rng = np.random.default_rng(seed)
        truth = rng.standard_normal((2, n))
        pad = max(1, max_shard(n, world))
        slabs = np.full((world, 2, pad), np.nan)
        ids = np.full((world, pad), -7, dtype=np.int32)
        for r in range(world):
            lo, hi = shard_bounds(n, r, world)
            perm = rng.permutation(hi - lo).astype(np.int32)  # slot s holds local particle perm[s]
            ids[r, : hi - lo] = perm
            slabs[r, :, : hi - lo] = truth[:, lo + perm]
        assert np.array_equal(unshard_slots(slabs, ids, n, world), truth)
        if n > 0:
            r = next(r for r in range(world) if shard_bounds(n, r, world)[1] > shard_bounds(n, r, world)[0])
            bad = ids.copy()
            bad[r, 0] = shard_bounds(n, r, world)[1] - shard_bounds(n, r, world)[0]
            with pytest.raises(ValueError):
                unshard_slots(slabs, bad, n, world)
            if shard_bounds(n, r, world)[1] - shard_bounds(n, r, world)[0] >= 2:
                dup = ids.copy()
                dup[r, 1] = dup[r, 0]  # a duplicated id would leave another particle's column unwritten
                with pytest.raises(ValueError):
                    unshard_slots(slabs, dup, n, world)
    prop()


def test_record_period_rules():
    import math
    from mops_amd.engine import TrajectoryConfig
    # streamline: run_time % recordT == 0, run_time = (j+1)*dt
    for dt, rt in ((120, 3600), (120, 300), (60, 90), (7, 3600)):
        per = rt // math.gcd(rt, dt)
        steps = [j for j in range(20000) if ((j + 1) * dt) % rt == 0]
        assert steps[:5] == [per * (i + 1) - 1 for i in range(5)]
    cfg = TrajectoryConfig(deltaT=60, simulationDuration=7 * 86400, recordT=3600)
    assert cfg.n_steps == 10080 and cfg.n_records == 168


def test_bench_bytes_model():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    # nv = 6 -> 3.66 kB (streamline L=60), 6.9 kB (pathline L=60), 8.8 kB (L=80)
    assert abs(bench.algorithmic_bytes_per_pstep(6, 60, 1) - 3660) < 5
    assert abs(bench.algorithmic_bytes_per_pstep(6, 60, 2) - 6924) < 50
    assert abs(bench.algorithmic_bytes_per_pstep(6, 80, 2) - 8844) < 50


def test_bench_roofline_uses_only_this_builds_pmc(tmp_path):
    """roofline.traffic/achieved/frac come from a PMC entry measured on this engine build only;
    a stale or missing entry gives nulls (advisor finding: round 1 read the committed traffic
    whatever kernel was built), and frac is a DRAM fraction, never the bytes model's."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    (tmp_path / "profiles").mkdir()
    key = "k"
    bid = bench.engine_build_id()
    bench.ROOT = str(tmp_path)
    assert bench.roofline_block("kern", 0.03, 7.2e8, 3660.0, key)["traffic"] is None  # no file
    pm = tmp_path / "profiles" / "pmc_traffic.json"
    pm.write_text(json.dumps([{"workload": key, "engine_build": "0" * 16, "bytes_per_unit": 5e9}]))
    r = bench.roofline_block("kern", 0.03, 7.2e8, 3660.0, key)
    assert r["traffic"] is None and r["frac"] is None and "stale" in r["traffic_source"]
    pm.write_text(json.dumps([{"workload": key, "engine_build": bid, "bytes_per_unit": 6e9,
                               "fp64_flops_per_unit": 6.0e11}]))
    r = bench.roofline_block("kern", 0.03, 7.2e8, 3660.0, key)
    assert r["traffic"] == 6e9 and abs(r["achieved"] - 200.0) < 1e-9 and abs(r["frac"] - 0.025) < 1e-12
    assert r["algorithmic_model"]["gbs"] > r["peak"]  # the model's rate is reported apart, not as frac
    assert abs(r["fp64_valu"]["achieved"] - 20.0) < 1e-9


# ---------------------------------------------------------------- gloo, world_size 2
def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from mops_amd import synth
        from mops_amd.distributed import max_shard, shard_bounds, unshard, unshard_slots
        from oracle import oracle as O
        mesh = synth.make_mesh(10, n_levels=8)
        s0 = synth.make_snapshot(mesh)
        d0 = O.preprocess(mesh, s0)
        seeds = synth.uniform_band_seeds(101, seed=9)
        lo, hi = shard_bounds(len(seeds), rank, world)
        npad = max_shard(len(seeds), world)
        r = O.run(mesh, d0, None, seeds[lo:hi], depth=200.0, delta_t=300, duration=10800, record_t=3600,
                  n_threads=1, finalize=False)
        K = r["rec_pos"].shape[1]
        slab = torch.zeros((K, 6, npad), dtype=torch.float64)
        slab[:, :3, : hi - lo] = torch.as_tensor(r["rec_pos"].transpose(1, 2, 0))
        slab[:, 3:, : hi - lo] = torch.as_tensor(r["rec_vel"].transpose(1, 2, 0))
        out = [torch.empty_like(slab) for _ in range(world)]
        dist.all_gather(out, slab)       # gloo has no all_gather_into_tensor on CPU for all versions
        full = unshard(torch.stack(out), len(seeds), world)
        # the GPU ranks' ParticleSet holds its records in slot (locality) order, slot s = local
        # particle ids[s]: gather slot-ordered slabs + ids and map them back (unshard_slots)
        g = torch.Generator().manual_seed(100 + rank)
        ids = torch.full((npad,), -1, dtype=torch.int32)
        ids[: hi - lo] = torch.randperm(hi - lo, generator=g).to(torch.int32)
        slot_slab = slab.clone()
        slot_slab[..., : hi - lo] = slab[..., ids[: hi - lo].long()]
        outs = [torch.empty_like(slot_slab) for _ in range(world)]
        outi = [torch.empty_like(ids) for _ in range(world)]
        dist.all_gather(outs, slot_slab)
        dist.all_gather(outi, ids)
        full_slots = unshard_slots(torch.stack(outs), torch.stack(outi), len(seeds), world)
        if rank == 0:
            ref = O.run(mesh, d0, None, seeds, depth=200.0, delta_t=300, duration=10800, record_t=3600,
                        n_threads=1, finalize=False)
            ok = all(np.array_equal(f[:, :3].numpy().transpose(2, 0, 1), ref["rec_pos"]) and
                     np.array_equal(f[:, 3:].numpy().transpose(2, 0, 1), ref["rec_vel"]) for f in (full, full_slots))
            q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_sharded_records_gloo_world2():
    import multiprocessing as mp
    import socket
    from oracle import oracle as O
    O.build()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


# ---------------------------------------------------------------- bench launcher / build identity
def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_bench_gpus_n_starts_its_own_ranks(monkeypatch):
    """`python bench.py --gpus N` (N > 1) with no launcher starts N ranks itself -- torch.distributed.run
    over 127.0.0.1 with the same arguments, as a child process (never exec) -- and exits with its status;
    under a launcher, a world size that differs from --gpus fails loudly."""
    import subprocess
    b = _bench()
    seen = {}

    class Done:
        returncode = 3

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2", "--backend", "gloo"])
    with pytest.raises(SystemExit) as e:
        b.main()
    assert e.value.code == 3
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == ["--gpus", "4", "--steps", "2", "--backend", "gloo"]
    assert os.path.samefile(cmd[-7], os.path.join(ROOT, "bench.py"))
    # launched by torchrun: WORLD_SIZE must equal --gpus
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:
        b.main()
    assert "--gpus 4" in str(e.value.code)
    b.check_world(2, 2)  # consistent: no error


def test_build_id_is_stamped_and_checked(engine_lib, tmp_path):
    """libmops_traj.so carries the build id of the sources next to it (mops_build_id), the loader
    refuses a library stamped with another id, and the id tracks every engine source and header."""
    import shutil
    from mops_amd import _build_id, _lib
    bid = _build_id.build_id()
    assert engine_lib.mops_build_id() == (_build_id.MARKER + bid).encode()
    assert _build_id.stamped_id(_lib.LIB_PATH) == bid
    assert len(_build_id.SOURCES) == 4 and all(os.path.exists(p) for p in _build_id.SOURCES + _build_id.HEADERS)
    # a stale library (other stamp) at the product path is refused
    stale = tmp_path / "libmops_traj.so"
    data = open(_lib.LIB_PATH, "rb").read().replace(bid.encode(), b"0" * 16)
    stale.write_bytes(data)
    saved_lib, saved_path = _lib._lib, _lib.LIB_PATH
    try:
        _lib._lib = None
        _lib.LIB_PATH = str(stale)
        with pytest.raises(_lib.MopsError, match="stale engine library"):
            _lib.load(str(stale))
    finally:
        _lib._lib, _lib.LIB_PATH = saved_lib, saved_path
    assert shutil.which("hipcc") is None or bid != _build_id.build_id(("-DMOPS_OTHER",))


def test_remove_nan_cpp_driver_compiles(engine_lib, tmp_path):
    """tests/cpp/remove_nan_api.cpp (the GPU test's C++ API driver) builds against the header and
    links against libmops_traj.so without a GPU."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    libdir = os.path.join(ROOT, "mops_amd", "lib")
    exe = str(tmp_path / "remove_nan_api")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "remove_nan_api.cpp"), "-L" + libdir, "-lmops_traj",
                    "-Wl,-rpath," + libdir, "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe], check=True)
    assert os.path.exists(exe)


def test_synth_library_rebuilds_by_build_id(tmp_path, monkeypatch):
    """libmops_synth.so (configs 4/5 snapshot generator) carries its source's id and is rebuilt when the
    stamp differs -- file times play no part (a stale library could otherwise feed configs 4/5)."""
    import shutil
    import __graft_entry__ as g
    from mops_amd import _build_id
    if shutil.which("hipcc") is None:
        pytest.skip("no hipcc")
    g.build_synth()
    assert _build_id.stamped_id(g.SYNTH_OUT) == g.synth_build_id()
    stale = tmp_path / "libmops_synth.so"
    stale.write_bytes(open(g.SYNTH_OUT, "rb").read().replace(g.synth_build_id().encode(), b"0" * 16))
    monkeypatch.setattr(g, "SYNTH_OUT", str(stale))
    calls = []
    real = g.subprocess.run
    monkeypatch.setattr(g.subprocess, "run", lambda cmd, **k: calls.append(cmd) or real(cmd, **k))
    g.build_synth()
    assert calls and _build_id.stamped_id(str(stale)) == g.synth_build_id()
