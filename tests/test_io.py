"""Trajectory output writers (include/mops_io.h): CLI txt dump, VTP polylines
with dateline splitting, and the pathline binary export -- checked by reading
the files back.  The writers are host code; only ``lines_geo`` needs a GPU."""
import json
import struct
import xml.etree.ElementTree as ET

import numpy as np
import pytest


def _geo_host(points, velocity):
    """GeoConverter::convertXYZToLatLonDegree + |v| (numpy restatement, test-only)."""
    x, y, z = points[..., 0], points[..., 1], points[..., 2]
    r = np.sqrt(x * x + y * y + z * z)
    lat = np.arcsin(z / r) * (180.0 / np.pi)
    lon = np.arctan2(y, x) * (180.0 / np.pi)
    vm = np.sqrt(velocity[..., 0] ** 2 + velocity[..., 1] ** 2 + velocity[..., 2] ** 2)
    return np.ascontiguousarray(np.stack([lat, lon, r, vm], axis=-1))


def _lines():
    from mops_amd import synth
    n, P = 3, 5
    lat = np.array([[10, 11, 12, 13, 14], [-5, -5, -5, -5, -5], [40, 41, 42, 43, 44]], dtype=float)
    lon = np.array([[0, 1, 2, 3, 4], [168, 172, 178, -179, -175], [-60, -61, -62, -63, -64]], dtype=float)
    pts = synth.latlon_to_xyz(lat, lon).reshape(n, P, 3)
    pts[2] *= 0.9999                                   # 637 m deeper
    rng = np.random.default_rng(1)
    vel = rng.normal(size=(n, P, 3)) * 0.1
    vel[:, -1] = 0.0
    tmp = rng.uniform(0, 30, (n, P)); sal = rng.uniform(30, 36, (n, P))
    return dict(points=pts, velocity=vel, temperature=tmp, salinity=sal)


def test_txt_dump(engine_lib, tmp_path):
    from mops_amd import io
    lines = _lines()
    f = tmp_path / "traj_line_0.txt"
    io.save_trajectory_lines_txt(str(f), lines)
    rows = f.read_text().splitlines()
    assert rows[0] == "Line_Index Point_Index Position_X Position_Y Position_Z Velocity_X Velocity_Y Velocity_Z"
    p, v = lines["points"], lines["velocity"]
    exp = [f"{l} {i} " + " ".join("%g" % x for x in (*p[l, i], *v[l, i])) for l in range(3) for i in range(5)]
    assert rows[1:] == exp


@pytest.mark.parametrize("binary", [False, True])
def test_vtp_polylines(engine_lib, tmp_path, binary):
    from mops_amd import io
    lines = _lines()
    geo = _geo_host(lines["points"], lines["velocity"])
    io.save_trajectory_lines_vtp(str(tmp_path / "traj"), lines, binary=binary, geo=geo)
    raw = (tmp_path / "traj.vtp").read_bytes()
    head, _, app = raw.partition(b"<AppendedData encoding=\"raw\">")
    root = ET.fromstring(head + (b"</VTKFile>" if binary else b""))
    piece = root.find("PolyData/Piece")
    assert piece.get("NumberOfPoints") == "15"
    assert piece.get("NumberOfLines") == "4"             # line 1 splits at the dateline (178 -> -179)
    arrays = {}
    blob = app[app.index(b"_") + 1:] if binary else b""
    for da in root.iter("DataArray"):
        dt = {"Float64": np.float64, "Float32": np.float32, "Int64": np.int64}[da.get("type")]
        if binary:
            off = int(da.get("offset"))
            nbytes = struct.unpack("<Q", blob[off:off + 8])[0]
            arrays[da.get("Name")] = np.frombuffer(blob[off + 8:off + 8 + nbytes], dtype=dt)
        else:
            arrays[da.get("Name")] = np.array(da.text.split(), dtype=dt)
    assert np.array_equal(arrays["offsets"], [5, 8, 10, 15])
    assert np.array_equal(arrays["connectivity"], np.arange(15))
    pts = arrays["Points"].reshape(-1, 3)
    exp = np.stack([geo[..., 1], geo[..., 0], 6371010.0 - geo[..., 2]], -1).reshape(-1, 3).astype(np.float32)
    assert np.array_equal(pts, exp)
    assert np.array_equal(arrays["temperature"], lines["temperature"].reshape(-1))
    assert np.array_equal(arrays["velocity_mag"], geo[..., 3].reshape(-1))


def test_pathline_binary_export(engine_lib, tmp_path):
    from mops_amd import io
    lines = _lines()
    geo = _geo_host(lines["points"], lines["velocity"])
    f = tmp_path / "paths.bin"
    io.export_pathlines_to_binary(lines, str(f), include_velocity=True, include_scalars=True, geo=geo)
    b = f.read_bytes()
    (n,) = struct.unpack_from("<i", b, 0)
    assert n == 3
    meta = json.loads((tmp_path / "paths.meta.json").read_text())
    assert meta["fields"] == ["lat", "lon", "velocity_u", "velocity_v", "speed", "temperature", "salinity"]
    off = 4
    for l in range(3):
        assert meta["particle_offsets"][l] == {"start": off, "points": 5}
        (m,) = struct.unpack_from("<i", b, off); off += 4
        rec = np.frombuffer(b, dtype="<f8", count=m * 7, offset=off).reshape(m, 7); off += m * 56
        assert np.array_equal(rec[:, 0], geo[l, :, 0]) and np.array_equal(rec[:, 1], geo[l, :, 1])
        assert np.array_equal(rec[:, 2:4], lines["velocity"][l, :, :2])
        assert np.array_equal(rec[:, 5], lines["temperature"][l]) and np.array_equal(rec[:, 6], lines["salinity"][l])
    assert off == len(b)


@pytest.mark.gpu
def test_lines_geo_device(engine_lib, gpu):
    from mops_amd import io
    lines = _lines()
    got = io.lines_geo(lines["points"], lines["velocity"]).cpu().numpy()
    ref = _geo_host(lines["points"], lines["velocity"])
    assert np.allclose(got, ref, rtol=1e-14, atol=1e-12)
