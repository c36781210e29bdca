"""MPAS-Ocean mesh / history ingest.

Mirrors the reference's MPASOReader (src/IO/MPASOReader.cpp:121-245) on top
of the native netCDF classic reader (include/mops_netcdf.h):

* the ftk stream YAML (tutorial/test.yaml): ``path_prefix``; substream 0 is
  the static mesh, substream 1 the time-varying data; ``filenames`` is a glob
  (sorted), and every listed variable is looked up by its ``possible_names``
  (or its ``name``) -- the value is stored under ``name``; a missing
  ``optional`` variable is skipped, any other missing variable is an error;
* ``readGridData(yaml)`` / ``readSolData(yaml, data_name, timestep)`` with the
  reference's file selection: the first data file whose name contains
  ``data_name``, global step = first_timestep_per_file[fi] + timestep;
* the reader's members carry the reference names (``cellCoord_vec``,
  ``verticesOnCell_vec``, ``cellLayerThickness_vec`` ...), so pyMOPS'
  ``init_from_reader`` and the engine's DeviceMesh/DeviceField take them as is.

netCDF-4/HDF5 files are rejected (MOPS_ERR_UNSUPPORTED): convert with
``nccopy -k cdf5``.
"""
from __future__ import annotations

import ctypes as C
import glob
import os
import types

import numpy as np

from . import _lib as L

_INT_TYPES = {1, 3, 4, 7, 8, 9, 10, 11}
_CHAR_TYPES = {2}


class NcFile:
    """One netCDF classic file (mops_nc_open)."""

    def __init__(self, path: str):
        self.lib = L.load()
        h = C.c_void_p()
        L.check(self.lib.mops_nc_open(path.encode(), C.byref(h)), f"mops_nc_open({path})")
        self.h = h
        self.path = path

    def close(self):
        if getattr(self, "h", None):
            self.lib.mops_nc_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def dim(self, name: str) -> int:
        v = C.c_int64()
        L.check(self.lib.mops_nc_dim_len(self.h, name.encode(), C.byref(v)), f"dimension {name}")
        return int(v.value)

    def info(self, name: str):
        """(type, shape, is_record) or None when the variable is absent."""
        t, nd, rec = C.c_int32(), C.c_int32(), C.c_int32()
        shape = (C.c_int64 * 8)()
        st = self.lib.mops_nc_var_info(self.h, name.encode(), C.byref(t), C.byref(nd), shape, C.byref(rec))
        if st != L.MOPS_OK:
            return None
        return int(t.value), tuple(int(shape[i]) for i in range(nd.value)), bool(rec.value)

    def read(self, name: str, record: int = 0) -> np.ndarray:
        t, shape, is_rec = self.info(name) or (None, None, None)
        if t is None:
            raise KeyError(f"{self.path}: no variable {name}")
        inner = shape[1:] if is_rec else shape
        count = int(np.prod(inner)) if inner else 1
        if t in _CHAR_TYPES:
            out = np.empty(count, dtype=np.uint8)
            fn = self.lib.mops_nc_read_bytes
        elif t in _INT_TYPES:
            out = np.empty(count, dtype=np.int64)
            fn = self.lib.mops_nc_read_i64
        else:
            out = np.empty(count, dtype=np.float64)
            fn = self.lib.mops_nc_read_f64
        L.check(fn(self.h, name.encode(), int(record) if is_rec else 0, out.ctypes.data_as(C.c_void_p), count),
                f"read {name}")
        return out.reshape(inner)


def _load_yaml(yaml_path: str) -> dict:
    import yaml
    with open(yaml_path) as f:
        return yaml.safe_load(f)["stream"]


def _files(stream: dict, sub: dict) -> list:
    names = sub["filenames"]
    names = names if isinstance(names, list) else [names]
    prefix = stream.get("path_prefix", "") or ""
    out = []
    for n in names:
        pat = n if os.path.isabs(n) else os.path.join(prefix, n)
        hits = sorted(glob.glob(pat))
        out.extend(hits if hits else [pat])
    return out


def _read_group(nc: NcFile, sub: dict, record: int) -> dict:
    group = {}
    for var in sub.get("vars", []) or []:
        name = var["name"]
        cands = var.get("possible_names") or [name]
        found = next((c for c in cands if nc.info(c) is not None), None)
        if found is None:
            if var.get("optional", False):
                continue
            raise KeyError(f"{nc.path}: none of {cands} present (variable '{name}')")
        group[name] = nc.read(found, record)
    return group


class MPASOReader:
    """Reference MPASOReader members, filled by readGridData / readSolData."""

    def __init__(self, yaml_path: str = ""):
        self.yaml_path = yaml_path
        self.mCellsSize = self.mEdgesSize = self.mMaxEdgesSize = self.mVertexSize = 0
        self.mVertLevels = self.mVertLevelsP1 = 0
        self.mTimesteps = 0
        self.mTimeStamp = ""
        self.mMeshName = self.mDataName = self.mFolderName = ""

    # ---- MPASOReader::readGridData (MPASOReader.cpp:128-169)
    @staticmethod
    def readGridData(yaml_path: str) -> "MPASOReader":
        stream = _load_yaml(yaml_path)
        sub = stream["substreams"][0]
        path = _files(stream, sub)[0]
        nc = NcFile(path)
        gs = _read_group(nc, sub, 0)
        r = MPASOReader(yaml_path)
        r.mMeshName = os.path.splitext(os.path.basename(path))[0]
        r.mFolderName = stream.get("path_prefix", "")

        def vec3(a, b, c):
            return np.stack([gs[a], gs[b], gs[c]], -1).astype(np.float64) if a in gs else np.empty((0, 3))

        def ints(name):
            return gs[name].astype(np.uint64).reshape(-1) if name in gs else np.empty(0, dtype=np.uint64)

        r.cellCoord_vec = vec3("xCell", "yCell", "zCell")
        r.vertexCoord_vec = vec3("xVertex", "yVertex", "zVertex")
        r.edgeCoord_vec = vec3("xEdge", "yEdge", "zEdge")
        r.verticesOnCell_vec = ints("verticesOnCell")
        r.verticesOnEdge_vec = ints("verticesOnEdge")
        r.cellsOnVertex_vec = ints("cellsOnVertex")
        r.cellsOnCell_vec = ints("cellsOnCell")
        r.numberVertexOnCell_vec = ints("nEdgesOnCell")
        r.cellsOnEdge_vec = ints("cellsOnEdge")
        r.edgesOnCell_vec = ints("edgesOnCell")
        r.cellRefBottomDepth_vec = gs["refBottomDepth"].astype(np.float64) if "refBottomDepth" in gs else np.empty(0)
        r.mCellsSize = len(r.cellCoord_vec)
        r.mEdgesSize = len(r.edgeCoord_vec)
        r.mVertexSize = len(r.vertexCoord_vec)
        per_cell = r.edgesOnCell_vec if r.edgesOnCell_vec.size else r.verticesOnCell_vec
        r.mMaxEdgesSize = per_cell.size // r.mCellsSize if r.mCellsSize else 0
        nc.close()
        return r

    @staticmethod
    def _locate(yaml_path: str, data_name: str, timestep: int):
        """(stream, data substream, file of the global step, record in it, the named file) -- the ftk
        stream's global step = first_timestep_per_file[file with data_name] + timestep."""
        if timestep < 0:
            raise ValueError(f"[MPASOReader]::Error: Invalid timestep index {timestep}")
        stream = _load_yaml(yaml_path)
        sub = stream["substreams"][1]
        files = _files(stream, sub)
        fi = next((i for i, f in enumerate(files) if data_name in os.path.basename(f) or data_name in f), None)
        if fi is None:
            raise FileNotFoundError(f"[MPASOReader]::Error: Data file with name containing '{data_name}' not found "
                                    f"in YAML.")
        counts = []
        for f in files:
            nc = NcFile(f)
            try:
                counts.append(nc.dim("Time"))
            except L.MopsError:
                counts.append(1)
            nc.close()
        first = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(int)
        index = int(first[fi]) + int(timestep)            # ftk stream->read(index)
        j = int(np.searchsorted(first, index, side="right") - 1)
        if j < 0 or index - first[j] >= counts[j]:
            raise IndexError(f"[MPASOReader]: global step {index} beyond the data files")
        return stream, sub, files[j], index - int(first[j]), files[fi]

    @staticmethod
    def readTimeStamp(yaml_path: str, data_name: str, timestep: int = 0) -> str:
        """The snapshot's xtime alone (what MPASOSolution::getTimeStamp returns after readSolData), without
        reading its fields: the chain needs every pair's gap before it derives any field."""
        _, sub, path, rec, _ = MPASOReader._locate(yaml_path, data_name, timestep)
        names = next((v.get("possible_names") or [v["name"]] for v in sub.get("vars", []) or []
                      if v["name"] == "xtime"), ["xtime", "xtime_startMonthly", "xtime_startDaily"])
        nc = NcFile(path)
        try:
            found = next((c for c in names if nc.info(c) is not None), None)
            if found is None:
                return ""
            return bytes(np.asarray(nc.read(found, rec), dtype=np.uint8).reshape(-1)).decode(errors="replace")
        finally:
            nc.close()

    # ---- MPASOReader::readSolData (MPASOReader.cpp:171-245)
    @staticmethod
    def readSolData(yaml_path: str, data_name: str, timestep: int = 0) -> "MPASOReader":
        stream, sub, path, rec, named = MPASOReader._locate(yaml_path, data_name, timestep)
        nc = NcFile(path)
        gs = _read_group(nc, sub, rec)
        nc.close()
        r = MPASOReader(yaml_path)
        r.mTimesteps = int(timestep)
        r.mDataName = os.path.splitext(os.path.basename(named))[0]
        r.mFolderName = stream.get("path_prefix", "")

        def d(name):
            return gs[name].astype(np.float64).reshape(-1) if name in gs else np.empty(0)

        r.cellBottomDepth_vec = d("bottomDepth")
        r.cellSurfaceHeight_vec = d("seaSurfaceHeight")
        r.cellZonalVelocity_vec = d("velocityZonal")
        r.cellMeridionalVelocity_vec = d("velocityMeridional")
        r.cellLayerThickness_vec = d("layerThickness")
        r.cellZTop_vec = d("zTop")
        r.cellNormalVelocity_vec = d("normalVelocity")
        r.cellVertVelocity_vec = d("vertVelocityTop")
        r.attributes = {k: d(k) for k in ("temperature", "salinity") if k in gs}
        xt = next((gs[k] for k in ("xtime", "xtime_startMonthly", "xtime_startDaily") if k in gs), None)
        r.mTimeStamp = bytes(np.asarray(xt, dtype=np.uint8).reshape(-1)).decode(errors="replace") if xt is not None \
            else ""
        if r.cellSurfaceHeight_vec.size:
            r.mVertLevels = r.cellLayerThickness_vec.size // r.cellSurfaceHeight_vec.size
        elif r.cellBottomDepth_vec.size:
            r.mVertLevels = r.cellLayerThickness_vec.size // r.cellBottomDepth_vec.size
        r.mVertLevelsP1 = r.mVertLevels + 1 if r.mVertLevels else 0
        return r


def mesh_from_reader(grid: MPASOReader, n_vert_levels: int):
    """Arrays DeviceMesh.from_mesh takes (MPASOGrid::initGrid, MPASOGrid.cpp:190-230)."""
    return types.SimpleNamespace(
        nCells=grid.mCellsSize, nVertices=grid.mVertexSize, maxEdges=grid.mMaxEdgesSize, nVertLevels=int(n_vert_levels),
        nEdgesOnCell=grid.numberVertexOnCell_vec, verticesOnCell=grid.verticesOnCell_vec,
        cellsOnCell=grid.cellsOnCell_vec, cellsOnVertex=grid.cellsOnVertex_vec, cellCoord=grid.cellCoord_vec,
        vertexCoord=grid.vertexCoord_vec)


def snapshot_from_reader(sol: MPASOReader, timestep_id: int | None = None):
    """Raw per-cell fields DeviceField.from_snapshot takes (MPASOSolution::initSolution)."""
    def opt(a):
        return a if a is not None and a.size else None
    return types.SimpleNamespace(
        timestep=sol.mTimesteps if timestep_id is None else int(timestep_id),
        layerThickness=opt(sol.cellLayerThickness_vec), bottomDepth=opt(sol.cellBottomDepth_vec),
        surfaceHeight=opt(sol.cellSurfaceHeight_vec), zonalVelocity=opt(sol.cellZonalVelocity_vec),
        meridionalVelocity=opt(sol.cellMeridionalVelocity_vec), vertVelocityTop=opt(sol.cellVertVelocity_vec))
