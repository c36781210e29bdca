"""MPAS netCDF ingest (mops_amd/mpas.py over include/mops_netcdf.h).

Fixtures are written here with scipy's netCDF3 writer (CDF-1 / CDF-2) and a
small CDF-5 writer below (test-only, following the published classic-format
spec), from a synthetic mesh laid out exactly like an MPAS restart/history
file: 1-based int32 connectivity, (Time, nCells, nVertLevels) records, xtime
as (Time, StrLen) chars, time-averaged names resolved via possible_names.
"""
import os
import struct

import numpy as np
import pytest

scipy_io = pytest.importorskip("scipy.io")


def _mesh():
    from mops_amd import synth
    mesh = synth.make_mesh(8, n_levels=6)
    snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.3 * t) for t in range(3)]
    return mesh, snaps


def _write_mesh(path, mesh, version):
    C, V, mE = mesh.nCells, mesh.nVertices, mesh.maxEdges
    f = scipy_io.netcdf_file(path, "w", version=version)
    f.createDimension("nCells", C); f.createDimension("nVertices", V)
    f.createDimension("maxEdges", mE); f.createDimension("vertexDegree", 3)
    f.createDimension("nVertLevels", mesh.nVertLevels)
    for k, a in zip("xyz", mesh.cellCoord.T):
        f.createVariable(f"{k}Cell", "d", ("nCells",))[:] = a
    for k, a in zip("xyz", mesh.vertexCoord.T):
        f.createVariable(f"{k}Vertex", "d", ("nVertices",))[:] = a
    f.createVariable("nEdgesOnCell", "i", ("nCells",))[:] = mesh.nEdgesOnCell.astype(np.int32)
    f.createVariable("verticesOnCell", "i", ("nCells", "maxEdges"))[:] = mesh.verticesOnCell.reshape(C, mE).astype(np.int32)
    f.createVariable("cellsOnCell", "i", ("nCells", "maxEdges"))[:] = mesh.cellsOnCell.reshape(C, mE).astype(np.int32)
    f.createVariable("cellsOnVertex", "i", ("nVertices", "vertexDegree"))[:] = mesh.cellsOnVertex.reshape(V, 3).astype(np.int32)
    f.createVariable("refBottomDepth", "d", ("nVertLevels",))[:] = mesh.refBottomDepth
    f.close()


def _write_hist(path, mesh, snaps, version, stamp0):
    C, L = mesh.nCells, mesh.nVertLevels
    f = scipy_io.netcdf_file(path, "w", version=version)
    f.createDimension("Time", None); f.createDimension("nCells", C)
    f.createDimension("nVertLevels", L); f.createDimension("nVertLevelsP1", L + 1); f.createDimension("StrLen", 64)
    xt = f.createVariable("xtime_startMonthly", "c", ("Time", "StrLen"))
    lt = f.createVariable("timeMonthly_avg_layerThickness", "d", ("Time", "nCells", "nVertLevels"))
    vz = f.createVariable("timeMonthly_avg_velocityZonal", "d", ("Time", "nCells", "nVertLevels"))
    vm = f.createVariable("timeMonthly_avg_velocityMeridional", "d", ("Time", "nCells", "nVertLevels"))
    vv = f.createVariable("timeMonthly_avg_vertVelocityTop", "d", ("Time", "nCells", "nVertLevelsP1"))
    bd = f.createVariable("bottomDepth", "d", ("nCells",))
    bd[:] = snaps[0].bottomDepth
    for t, s in enumerate(snaps):
        xt[t] = np.frombuffer(f"{stamp0 + t:04d}-01-01_00:00:00".ljust(64).encode(), dtype="S1")
        lt[t] = s.layerThickness.reshape(C, L)
        vz[t] = s.zonalVelocity.reshape(C, L)
        vm[t] = s.meridionalVelocity.reshape(C, L)
        vv[t] = s.vertVelocityTop.reshape(C, L + 1)
    f.close()


YAML = """stream:
  name: mpas
  path_prefix: "{prefix}"
  substreams:
    - name: mesh
      format: netcdf
      filenames: "mesh.nc"
      static: true
      vars:
        - name: xCell
        - name: yCell
        - name: zCell
        - name: xVertex
        - name: yVertex
        - name: zVertex
        - name: nEdgesOnCell
        - name: cellsOnCell
        - name: cellsOnVertex
        - name: verticesOnCell
        - name: refBottomDepth
    - name: data
      format: netcdf
      filenames: "hist.am.timeSeriesStatsMonthly.*.nc"
      vars:
        - name: xtime
          possible_names: [xtime, xtime_startMonthly]
        - name: velocityZonal
          possible_names: [velocityZonal, timeMonthly_avg_velocityZonal]
        - name: velocityMeridional
          possible_names: [velocityMeridional, timeMonthly_avg_velocityMeridional]
        - name: vertVelocityTop
          possible_names: [vertVelocityTop, timeMonthly_avg_vertVelocityTop]
        - name: layerThickness
          possible_names: [layerThickness, timeMonthly_avg_layerThickness]
        - name: salinity
          possible_names: [salinity, timeMonthly_avg_activeTracers_salinity]
          optional: true
        - name: bottomDepth
          possibel_names: [bottomDepth]
"""


@pytest.mark.parametrize("version", [1, 2])
def test_mpas_reader_classic(engine_lib, tmp_path, version):
    from mops_amd.mpas import MPASOReader, mesh_from_reader, snapshot_from_reader
    mesh, snaps = _mesh()
    _write_mesh(str(tmp_path / "mesh.nc"), mesh, version)
    _write_hist(str(tmp_path / "hist.am.timeSeriesStatsMonthly.0001-01-01.nc"), mesh, snaps[:2], version, 1)
    _write_hist(str(tmp_path / "hist.am.timeSeriesStatsMonthly.0001-02-01.nc"), mesh, snaps[2:], version, 3)
    y = tmp_path / "mpas.yaml"
    y.write_text(YAML.format(prefix=str(tmp_path)))
    g = MPASOReader.readGridData(str(y))
    assert (g.mCellsSize, g.mVertexSize, g.mMaxEdgesSize) == (mesh.nCells, mesh.nVertices, mesh.maxEdges)
    assert np.array_equal(g.cellCoord_vec, mesh.cellCoord) and np.array_equal(g.vertexCoord_vec, mesh.vertexCoord)
    for a, b in ((g.verticesOnCell_vec, mesh.verticesOnCell), (g.cellsOnCell_vec, mesh.cellsOnCell),
                 (g.cellsOnVertex_vec, mesh.cellsOnVertex), (g.numberVertexOnCell_vec, mesh.nEdgesOnCell)):
        assert a.dtype == np.uint64 and np.array_equal(a, b)
    assert np.array_equal(g.cellRefBottomDepth_vec, mesh.refBottomDepth)
    # second file, first record: global step = first_timestep_per_file[1] + 0 = 2
    s = MPASOReader.readSolData(str(y), "0001-02-01", 0)
    assert s.mVertLevels == mesh.nVertLevels and s.mVertLevelsP1 == mesh.nVertLevels + 1
    assert s.mTimeStamp.startswith("0003-01-01_00:00:00")
    # the xtime alone (MOPSPathline reads every snapshot's stamp before deriving any field)
    assert MPASOReader.readTimeStamp(str(y), "0001-02-01", 0) == s.mTimeStamp
    assert MPASOReader.readTimeStamp(str(y), "0001-01-01", 1).startswith("0002-01-01_00:00:00")
    assert np.array_equal(s.cellLayerThickness_vec, snaps[2].layerThickness)
    assert np.array_equal(s.cellZonalVelocity_vec, snaps[2].zonalVelocity)
    assert np.array_equal(s.cellVertVelocity_vec, snaps[2].vertVelocityTop)
    assert np.array_equal(s.cellBottomDepth_vec, snaps[0].bottomDepth)
    # first file, record 1 ("possible_names" resolution, time index inside a file)
    s1 = MPASOReader.readSolData(str(y), "0001-01-01", 1)
    assert np.array_equal(s1.cellMeridionalVelocity_vec, snaps[1].meridionalVelocity)
    m = mesh_from_reader(g, s.mVertLevels)
    sn = snapshot_from_reader(s)
    assert m.nVertLevels == mesh.nVertLevels and sn.surfaceHeight is None
    with pytest.raises(FileNotFoundError):
        MPASOReader.readSolData(str(y), "9999-01-01", 0)


def test_pymops_init_from_reader(engine_lib, tmp_path):
    from mops_amd import pyMOPS
    mesh, snaps = _mesh()
    _write_mesh(str(tmp_path / "mesh.nc"), mesh, 2)
    _write_hist(str(tmp_path / "hist.am.timeSeriesStatsMonthly.0001-01-01.nc"), mesh, snaps[:2], 2, 1)
    y = tmp_path / "mpas.yaml"
    y.write_text(YAML.format(prefix=str(tmp_path)))
    grid = pyMOPS.MPASOGrid()
    grid.init_from_reader(pyMOPS.MPASOReader.readGridData(str(y)))
    a, b = pyMOPS.MPASOSolution(), pyMOPS.MPASOSolution()
    a.init_from_reader(pyMOPS.MPASOReader.readSolData(str(y), "0001-01-01", 0))
    b.init_from_reader(pyMOPS.MPASOReader.readSolData(str(y), "0001-01-01", 1))
    assert a.getID() != b.getID()                 # distinct xtime stamps -> distinct FNV-1a ids
    assert grid.mCellsSize == mesh.nCells and a.mVertLevels == mesh.nVertLevels


# ---- CDF-5 (64-bit data) writer: header per the classic-format spec, big endian
def _cdf5(path, dims, variables, numrecs):
    """dims: [(name, len or 0 for unlimited)]; variables: [(name, dimids, nc_type, ndarray)]."""
    def i64(v): return struct.pack(">q", v)
    def i32(v): return struct.pack(">i", v)
    def name(s):
        b = s.encode(); return i64(len(b)) + b + b"\0" * ((4 - len(b) % 4) % 4)
    tsz = {4: 4, 6: 8, 10: 8}
    hdr = b"CDF\x05" + i64(numrecs) + i32(10) + i64(len(dims))
    for n, l in dims:
        hdr += name(n) + i64(l)
    hdr += i32(0) + i64(0)                                       # no global attributes
    rec_dim = next(i for i, (_, l) in enumerate(dims) if l == 0)

    def var_bytes(v):
        nm, ids, t, a = v
        inner = [dims[i][1] for i in ids if i != rec_dim]
        return int(np.prod(inner)) * tsz[t], ids and ids[0] == rec_dim

    def header(begins):
        h = hdr + i32(11) + i64(len(variables))
        for (nm, ids, t, a), b in zip(variables, begins):
            sz, _ = var_bytes((nm, ids, t, a))
            h += name(nm) + i64(len(ids)) + b"".join(i64(i) for i in ids) + i32(0) + i64(0) + i32(t) + i64(sz) + i64(b)
        return h
    hlen = len(header([0] * len(variables)))
    fixed = [v for v in variables if not var_bytes(v)[1]]
    recs = [v for v in variables if var_bytes(v)[1]]
    begins, off = {}, hlen
    for v in fixed:
        begins[v[0]] = off; off += var_bytes(v)[0]
    for v in recs:
        begins[v[0]] = off; off += var_bytes(v)[0]
    body = b""
    fmt = {4: ">i4", 6: ">f8", 10: ">i8"}
    for v in fixed:
        body += np.asarray(v[3], dtype=fmt[v[2]]).tobytes()
    for r in range(numrecs):
        for v in recs:
            body += np.asarray(v[3][r], dtype=fmt[v[2]]).tobytes()
    with open(path, "wb") as f:
        f.write(header([begins[v[0]] for v in variables]) + body)


def test_cdf5_reader(engine_lib, tmp_path):
    from mops_amd.mpas import NcFile
    rng = np.random.default_rng(0)
    a = rng.normal(size=(5, 7)); ids = rng.integers(-2**40, 2**40, size=5)
    rec = rng.normal(size=(3, 5, 2)); rid = rng.integers(0, 100, size=(3, 5)).astype(np.int32)
    p = str(tmp_path / "x.nc")
    _cdf5(p, [("Time", 0), ("nCells", 5), ("nLev", 7), ("two", 2)],
          [("a", [1, 2], 6, a), ("ids", [1], 10, ids), ("rec", [0, 1, 3], 6, rec), ("rid", [0, 1], 4, rid)], 3)
    nc = NcFile(p)
    assert nc.dim("Time") == 3 and nc.dim("nLev") == 7
    assert np.array_equal(nc.read("a"), a) and np.array_equal(nc.read("ids"), ids)
    for r in range(3):
        assert np.array_equal(nc.read("rec", r), rec[r]) and np.array_equal(nc.read("rid", r), rid[r])
    assert nc.info("missing") is None


def test_hdf5_rejected(engine_lib, tmp_path):
    from mops_amd import _lib
    from mops_amd.mpas import NcFile
    p = tmp_path / "h.nc"
    p.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(_lib.MopsError, match="HDF5"):
        NcFile(str(p))
