"""mops_write_pathline_binary pinned by the reference's own exporter.

tests/golden/pathline_binary_* are the outputs of the reference's
tutorial/export_pathline_binary.py (``export_pathlines_to_binary``) on fixed
pathlines (generator: tests/golden/make_pathline_binary.py, run in the build
container only).

* CPU: given the reference's own lat/lon/speed arithmetic (numpy, the same
  process), the native writer reproduces the .bin and .meta.json files byte
  for byte -- header, per-particle counts, field order, offsets, JSON layout.
* GPU: with lat/lon/speed computed on the device (mops_lines_geo, the
  product path), every integer, every copied double (velocity_u/v,
  temperature, salinity) is bit-identical and lat/lon/speed are within
  4 ulp.  Tolerance: numpy evaluates arcsin/arctan2 with its own SIMD kernels
  (AVX-512 SVML here) and the speed with OpenBLAS ddot, which already differ
  from glibc by up to 1 ulp (asin/atan2) and 2 ulp (norm) on this host
  (measured over 2e6 arguments); device asin/atan2 are the ROCm device
  library's, so the reference's own result is CPU-dependent at the last ulp.
"""
import json
import os
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
TAGS = {"plain": (False, False), "vel": (True, False), "vel_scalars": (True, True)}
ULP_TOL = 4


def _inputs():
    g = np.load(os.path.join(GOLDEN, "pathline_binary_inputs.npz"))
    return {k: g[k] for k in ("points", "velocity", "temperature", "salinity")}


def _parse(raw, nfields):
    n = struct.unpack_from("<i", raw, 0)[0]
    pos, counts, rows = 4, [], []
    for _ in range(n):
        P = struct.unpack_from("<i", raw, pos)[0]; pos += 4
        counts.append(P)
        rows.append(np.frombuffer(raw, dtype="<f8", count=P * nfields, offset=pos).reshape(P, nfields))
        pos += 8 * P * nfields
    assert pos == len(raw)
    return n, counts, rows


def _write(tmp_path, tag, geo, inp):
    import ctypes as C
    from mops_amd import _lib
    lib = _lib.load()
    vel_on, sca_on = TAGS[tag]
    n, P = inp["points"].shape[:2]
    g = np.ascontiguousarray(geo, dtype=np.float64)
    v = np.ascontiguousarray(inp["velocity"], dtype=np.float64)
    t = np.ascontiguousarray(inp["temperature"], dtype=np.float64)
    s = np.ascontiguousarray(inp["salinity"], dtype=np.float64)
    path = str(tmp_path / f"pathline_binary_{tag}.bin")
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    _lib.check(lib.mops_write_pathline_binary(path.encode(), n, P, p(g), p(v), p(t), p(s), int(vel_on), int(sca_on)),
               "mops_write_pathline_binary")
    return open(path, "rb").read(), open(str(tmp_path / f"pathline_binary_{tag}.meta.json"), "rb").read()


def _golden(tag):
    return (open(os.path.join(GOLDEN, f"pathline_binary_{tag}.bin"), "rb").read(),
            open(os.path.join(GOLDEN, f"pathline_binary_{tag}.meta.json"), "rb").read())


def _reference_geo(inp):
    """export_pathline_binary.py:17-23 + :102 arithmetic, vectorised the same way (numpy)."""
    pts, vel = inp["points"], inp["velocity"]
    n, P = pts.shape[:2]
    geo = np.empty((n, P, 4))
    for i in range(n):
        x, y, z = pts[i, :, 0], pts[i, :, 1], pts[i, :, 2]
        lon = np.degrees(np.arctan2(y, x))
        r = np.sqrt(x * x + y * y + z * z)
        lat = np.degrees(np.arcsin(z / r))
        geo[i, :, 0], geo[i, :, 1], geo[i, :, 2] = lat, lon, r
        geo[i, :, 3] = [np.linalg.norm(vel[i, j]) for j in range(P)]
    return geo


@pytest.mark.parametrize("tag", list(TAGS))
def test_pathline_binary_writer_bytes(engine_lib, tmp_path, tag):
    """The writer's byte layout equals the reference exporter's, given the same doubles."""
    inp = _inputs()
    b, m = _write(tmp_path, tag, _reference_geo(inp), inp)
    gb, gm = _golden(tag)
    assert m == gm, "meta.json differs from export_pathline_binary.py's"
    assert b == gb, "binary differs from export_pathline_binary.py's"


def _ulps(a, b):
    a = np.asarray(a, dtype=np.float64); b = np.asarray(b, dtype=np.float64)
    ia, ib = a.view(np.int64), b.view(np.int64)
    ia = np.where(ia < 0, np.int64(-2**63) - ia, ia); ib = np.where(ib < 0, np.int64(-2**63) - ib, ib)
    return np.abs(ia - ib)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", list(TAGS))
def test_pathline_binary_device_geo_vs_reference(gpu, engine_lib, tmp_path, tag):
    """Product path: lat/lon/r/|v| from mops_lines_geo on the device, then the native writer."""
    import ctypes as C
    import torch
    from mops_amd import _lib
    inp = _inputs()
    n, P = inp["points"].shape[:2]
    dev = torch.device("cuda", 0)
    dp = torch.as_tensor(inp["points"], device=dev).contiguous()
    dv = torch.as_tensor(inp["velocity"], device=dev).contiguous()
    dg = torch.empty((n, P, 4), dtype=torch.float64, device=dev)
    _lib.check(engine_lib.mops_lines_geo(n, P, C.c_void_p(dp.data_ptr()), C.c_void_p(dv.data_ptr()),
                                         C.c_void_p(dg.data_ptr()), None), "mops_lines_geo")
    torch.cuda.synchronize()
    b, m = _write(tmp_path, tag, dg.cpu().numpy(), inp)
    gb, gm = _golden(tag)
    assert m == gm
    assert len(b) == len(gb)
    nf = 2 + (3 if TAGS[tag][0] else 0) + (2 if TAGS[tag][1] else 0)
    n1, c1, r1 = _parse(b, nf)
    n2, c2, r2 = _parse(gb, nf)
    assert (n1, c1) == (n2, c2)
    approx = [0, 1] + ([4] if TAGS[tag][0] else [])           # lat, lon, speed
    exact = [f for f in range(nf) if f not in approx]         # velocity_u/v, temperature, salinity: copies
    worst = 0
    for a, g in zip(r1, r2):
        assert np.array_equal(a[:, exact], g[:, exact])
        worst = max(worst, int(_ulps(a[:, approx], g[:, approx]).max()))
    assert worst <= ULP_TOL, f"lat/lon/speed differ from the reference exporter by {worst} ulp"
