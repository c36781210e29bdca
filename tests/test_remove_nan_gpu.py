"""The shipped HIP RemoveNaN paths pinned by the reference's own vectors.

test/test_trajector.cpp:26-194 holds the only golden vectors of the trajectory
output path: four RemoveNaNTrajectoriesAndReindex cases (tests/golden/
remove_nan_cases.json, made by tests/golden/make_golden.py).  Here they run
through every product entry point that cleans lines on the device:

  * mops_remove_nan_ragged -- all cases packed into ONE launch (ragged lengths
    4, 4, 5, 4, plus an empty line and a line whose velocity is shorter than
    its points, which the reference resizes with zeros, TrajectoryCommon.h:88);
  * mops_remove_nan_lines -- each case as a uniform batch;
  * MOPS::RemoveNaNTrajectoriesAndReindex (the C++ API) through a compiled
    driver, which also checks the reference's drop-empty-and-reindex rule.

Every case is compared with its full expected arrays (NaN patterns included),
which covers the reference test's asserted subset ("asserted" in the JSON).
"""
import json
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "remove_nan_cases.json")


def _cases():
    return json.load(open(GOLDEN))["cases"]


def _same(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(np.nan_to_num(a),
                                                                                             np.nan_to_num(b))


def _check(case, pts, vel, tmp, sal, last):
    e = case["expected"]
    assert set(case["asserted"]) <= {"len", "lineID", "points", "points.x", "points.x_is_nan", "points[0:2]",
                                     "points[2:]", "velocity", "velocity[1:]", "lastPoint", "lastPoint.xy"}
    assert len(pts) == len(e["points"]), case["name"]                     # original length preserved
    assert _same(pts, e["points"]), case["name"]
    assert _same(vel, e["velocity"]), case["name"]
    assert _same(tmp, e["temperature"]) and _same(sal, e["salinity"]), case["name"]
    assert _same(last, e["lastPoint"]), case["name"]


def _extra_lines(oracle_lib):
    """Ragged extras beyond the reference's four: a line whose velocity vector is two entries
    short (resized with zeros, :88) and an empty line (dropped, :84-86); expectations from the
    oracle restatement of the same function."""
    rng = np.random.default_rng(7)
    p = rng.normal(size=(6, 3)) * 1e6
    p[4, 2] = np.inf
    v_short = rng.normal(size=(4, 3))
    t = rng.normal(size=6); s = rng.normal(size=6)
    v_full = np.concatenate([v_short, np.zeros((2, 3))])
    e_pts, e_vel, e_tmp, e_sal, e_last = oracle_lib.remove_nan(p, v_full, t, s)
    short = dict(points=p, velocity=v_short, temperature=t, salinity=s,
                 expected=dict(points=e_pts, velocity=e_vel, temperature=e_tmp, salinity=e_sal, lastPoint=e_last))
    empty = dict(points=np.zeros((0, 3)), velocity=np.zeros((0, 3)), temperature=np.zeros(0), salinity=np.zeros(0))
    return short, empty


def _lib():
    from mops_amd import _lib
    return _lib


def test_remove_nan_ragged_one_launch(gpu, engine_lib, oracle_lib):
    """All reference cases + the extras cleaned by a single mops_remove_nan_ragged launch."""
    import ctypes as C
    import torch
    L = _lib()
    cases = _cases()
    short, empty = _extra_lines(oracle_lib)
    lines = [dict(points=np.array(c["input"]["points"], dtype=np.float64),
                  velocity=np.array(c["input"]["velocity"], dtype=np.float64),
                  temperature=np.array(c["input"]["temperature"], dtype=np.float64),
                  salinity=np.array(c["input"]["salinity"], dtype=np.float64)) for c in cases]
    lines.insert(2, empty)
    lines.append(short)
    off = np.zeros(len(lines) + 1, dtype=np.int64)
    for i, l in enumerate(lines):
        off[i + 1] = off[i] + len(l["points"])
    T = int(off[-1])
    pts = np.concatenate([l["points"] for l in lines])
    vel = np.concatenate([np.concatenate([l["velocity"], np.zeros((len(l["points"]) - len(l["velocity"]), 3))])
                          for l in lines])  # the resize the host does before packing (:88)
    tmp = np.concatenate([l["temperature"] for l in lines]); sal = np.concatenate([l["salinity"] for l in lines])
    dev = torch.device("cuda", 0)
    d = {k: torch.as_tensor(a, device=dev).contiguous() for k, a in
         dict(pts=pts, vel=vel, tmp=tmp, sal=sal, off=off).items()}
    last = torch.full((len(lines), 3), -7.0, dtype=torch.float64, device=dev)
    rc = engine_lib.mops_remove_nan_ragged(len(lines), C.c_void_p(d["off"].data_ptr()), C.c_void_p(d["pts"].data_ptr()),
                                           C.c_void_p(d["vel"].data_ptr()), C.c_void_p(d["tmp"].data_ptr()),
                                           C.c_void_p(d["sal"].data_ptr()), C.c_void_p(last.data_ptr()), None)
    L.check(rc, "mops_remove_nan_ragged")
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in d.items()}
    lastn = last.cpu().numpy()
    exp = [c for c in cases]
    exp.insert(2, None)
    exp.append(dict(name="short_velocity", asserted=[], expected=short["expected"]))
    assert T == sum(len(l["points"]) for l in lines)
    for i, c in enumerate(exp):
        a, b = off[i], off[i + 1]
        if c is None:  # the empty line is untouched (its last point too)
            assert b == a and np.all(lastn[i] == -7.0)
            continue
        _check(c, got["pts"][a:b], got["vel"][a:b], got["tmp"][a:b], got["sal"][a:b], lastn[i])


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c["name"])
def test_remove_nan_uniform_lines(gpu, engine_lib, case):
    """Each reference case through mops_remove_nan_lines (uniform batch of 3 copies)."""
    import ctypes as C
    import torch
    L = _lib()
    inp = case["input"]
    P = len(inp["points"])
    dev = torch.device("cuda", 0)
    rep = lambda a: torch.as_tensor(np.stack([np.array(a, dtype=np.float64)] * 3), device=dev).contiguous()
    pts, vel, tmp, sal = rep(inp["points"]), rep(inp["velocity"]), rep(inp["temperature"]), rep(inp["salinity"])
    last = torch.empty((3, 3), dtype=torch.float64, device=dev)
    L.check(engine_lib.mops_remove_nan_lines(3, P, C.c_void_p(pts.data_ptr()), C.c_void_p(vel.data_ptr()),
                                             C.c_void_p(tmp.data_ptr()), C.c_void_p(sal.data_ptr()),
                                             C.c_void_p(last.data_ptr()), None), "mops_remove_nan_lines")
    torch.cuda.synchronize()
    for j in range(3):
        _check(case, pts[j].cpu().numpy(), vel[j].cpu().numpy(), tmp[j].cpu().numpy(), sal[j].cpu().numpy(),
               last[j].cpu().numpy())


def _compile_driver(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = os.path.join(str(tmp_path), "remove_nan_api")
    libdir = os.path.join(ROOT, "mops_amd", "lib")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "remove_nan_api.cpp"), "-L" + libdir, "-lmops_traj",
                    "-Wl,-rpath," + libdir, "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe], check=True)
    return exe


def test_cpp_api_remove_nan_reindex(gpu, engine_lib, oracle_lib, tmp_path):
    """MOPS::RemoveNaNTrajectoriesAndReindex on the reference cases in one call (+ an empty line,
    dropped, and a short-velocity line): the reference test's assertions, lineIDs re-numbered."""
    exe = _compile_driver(tmp_path)
    cases = _cases()
    short, empty = _extra_lines(oracle_lib)
    ins = [dict(points=c["input"]["points"], velocity=c["input"]["velocity"], temperature=c["input"]["temperature"],
                salinity=c["input"]["salinity"], lineID=c["input"]["lineID"]) for c in cases]
    ins.insert(1, dict(empty, lineID=5))
    ins.append(dict(short, lineID=9))
    with open(tmp_path / "in.bin", "wb") as f:
        f.write(struct.pack("<q", len(ins)))
        for l in ins:
            p = np.asarray(l["points"], dtype=np.float64).reshape(-1, 3)
            v = np.asarray(l["velocity"], dtype=np.float64).reshape(-1, 3)
            f.write(struct.pack("<qqq", int(l["lineID"]), len(p), len(v)))
            for a in (p, v, l["temperature"], l["salinity"]):
                f.write(np.ascontiguousarray(a, dtype="<f8").tobytes())
    r = subprocess.run([exe, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    raw = open(tmp_path / "out.bin", "rb").read()
    m = struct.unpack_from("<q", raw, 0)[0]
    pos = 8
    exp = cases + [dict(name="short_velocity", asserted=[], expected=short["expected"])]
    assert m == len(exp)  # the empty line is dropped (TrajectoryCommon.h:84-86)
    for i in range(m):
        lid, P = struct.unpack_from("<qq", raw, pos); pos += 16
        a = np.frombuffer(raw, dtype="<f8", count=P * 8, offset=pos).reshape(P, 8); pos += P * 64
        last = np.frombuffer(raw, dtype="<f8", count=3, offset=pos); pos += 24
        assert lid == i  # re-indexed in order (:124)
        _check(exp[i], a[:, 0:3], a[:, 3:6], a[:, 6], a[:, 7], last)
