"""pyMOPS-compatible Python API for the MI355X trajectory engine.

Mirrors the trajectory surface of the reference's pybind module
(tools/pyMOPS/bindings.cpp:23-455): the same enum, class and function names,
the same argument meaning and the same return layout, so a pyMOPS script's
trajectory part runs unchanged with ``from mops_amd import pyMOPS``:

    MOPS_Init / MOPS_Begin / MOPS_AddGridMesh / MOPS_AddAttribute / MOPS_End /
    MOPS_ActiveAttribute                       (bindings.cpp:281-286)
    MOPS_GenerateSeedsPoints(SeedsSettings)    -> (N, 3) float64   (:311-327)
    MOPS_RunStreamLine(cfg, (N, 3))            -> [ {lineID, points, velocity} ]           (:328-381)
    MOPS_RunPathLine(cfg, (N, 3))              -> [ {lineID, points, velocity, temperature,
                                                     salinity, lastPoint, depth} ]          (:383-455)
    MOPS_ResetTiming / MOPS_PrintTimingSummary / MOPS_PrintTimingDetailed /
    MOPS_GetCategoryTime / MOPS_GetTotalTime   (:457-475)

Every trajectory goes through the HIP engine (``engine.run_trajectories`` on
the C ABI); there is no CPU path.  ``MPASOReader`` / ``init_from_reader``
load MPAS netCDF classic files (mops_amd/mpas.py).  Out of scope:
image remapping (``MOPS_RunRemapping`` / ``MOPS_RunReGrid``) raises
``NotImplementedError``.
"""
from __future__ import annotations

import enum
import math
import sys
import time
import types

import numpy as np

from . import engine as _E
from . import _lib as _L
from .mpas import MPASOReader  # noqa: F401  (bindings.cpp:88-91: readGridData / readSolData)


class CalcDirection(enum.IntEnum):
    kForward = 0
    kBackward = 1


class CalcMethodType(enum.IntEnum):
    kRK4 = 0
    kEuler = 1


class GridAttributeType(enum.IntEnum):
    kCellSize = 0
    kEdgeSize = 1
    kVertexSize = 2
    kMaxEdgesSize = 3
    kVertLevels = 4
    kVertLevelsP1 = 5
    kVertexCoord = 6
    kCellCoord = 7
    kEdgeCoord = 8
    kVertexLatLon = 9
    kVerticesOnCell = 10
    kVerticesOnEdge = 11
    kCellsOnVertex = 12
    kCellsOnCell = 13
    kNumberVertexOnCell = 14
    kCellsOnEdge = 15
    kEdgesOnCell = 16
    kCellWeight = 17


class AttributeType(enum.IntEnum):
    kZonalVelocity = 0
    kMeridionalVelocity = 1
    kVelocity = 2
    kNormalVelocity = 3
    kZTop = 4
    kLayerThickness = 5
    kBottomDepth = 6


def _error(msg: str):
    print(f"[Error]: {msg}", file=sys.stderr)


# ---- data model (MPASOGrid.cpp:82-188, MPASOSolution.cpp:1145-1210) -------

_GRID_SCALARS = {GridAttributeType.kCellSize: "mCellsSize", GridAttributeType.kEdgeSize: "mEdgesSize",
                 GridAttributeType.kVertexSize: "mVertexSize", GridAttributeType.kMaxEdgesSize: "mMaxEdgesSize",
                 GridAttributeType.kVertLevels: "mVertLevels", GridAttributeType.kVertLevelsP1: "mVertLevelsP1"}


class MPASOGrid:
    def __init__(self):
        self.mCellsSize = self.mEdgesSize = self.mMaxEdgesSize = self.mVertexSize = 0
        self.mVertLevels = self.mVertLevelsP1 = 0
        self.vec3 = {}
        self.ints = {}

    def init_from_reader(self, reader):
        """MPASOGrid::initGrid(MPASOReader*) (MPASOGrid.cpp:190-230)."""
        G = GridAttributeType
        self.mCellsSize, self.mEdgesSize = reader.mCellsSize, reader.mEdgesSize
        self.mMaxEdgesSize, self.mVertexSize = reader.mMaxEdgesSize, reader.mVertexSize
        self.mVertLevels, self.mVertLevelsP1 = reader.mVertLevels, reader.mVertLevelsP1
        self.vec3 = {G.kCellCoord: reader.cellCoord_vec, G.kVertexCoord: reader.vertexCoord_vec,
                     G.kEdgeCoord: reader.edgeCoord_vec}
        self.ints = {G.kVerticesOnCell: reader.verticesOnCell_vec, G.kVerticesOnEdge: reader.verticesOnEdge_vec,
                     G.kCellsOnVertex: reader.cellsOnVertex_vec, G.kCellsOnCell: reader.cellsOnCell_vec,
                     G.kNumberVertexOnCell: reader.numberVertexOnCell_vec, G.kCellsOnEdge: reader.cellsOnEdge_vec,
                     G.kEdgesOnCell: reader.edgesOnCell_vec}

    def init_from_yaml(self, yaml_path):
        """MPASOGrid::initGrid_DemoLoading (MPASOGrid.cpp:14-27)."""
        self.init_from_reader(MPASOReader.readGridData(yaml_path))

    def setGridAttribute(self, type, val: int):
        name = _GRID_SCALARS.get(GridAttributeType(type))
        if name is None:
            _error("[MPASOGrid]::Invalid GridAttributeType")
            return
        setattr(self, name, int(val))

    def setGridAttributesVec3(self, type, arr):
        type = GridAttributeType(type)
        if type not in (GridAttributeType.kVertexCoord, GridAttributeType.kCellCoord, GridAttributeType.kEdgeCoord):
            print("Error: Invalid GridAttributeType")
            return
        self.vec3[type] = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1, 3)

    def setGridAttributesVec2(self, type, arr):
        if GridAttributeType(type) != GridAttributeType.kVertexLatLon:
            print("Error: Invalid GridAttributeType")
            return
        self.vertexLatLon = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1, 2)

    def setGridAttributesInt(self, type, arr):
        self.ints[GridAttributeType(type)] = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1)

    def setGridAttributesFloat(self, type, arr):
        self.cellWeight = np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)

    def checkAttribute(self) -> bool:
        need_i = (GridAttributeType.kVerticesOnCell, GridAttributeType.kCellsOnVertex, GridAttributeType.kCellsOnCell,
                  GridAttributeType.kNumberVertexOnCell)
        return (self.mCellsSize and self.mVertexSize and self.mMaxEdgesSize and self.mVertLevels
                and GridAttributeType.kCellCoord in self.vec3 and GridAttributeType.kVertexCoord in self.vec3
                and all(t in self.ints for t in need_i))


class MPASOSolution:
    def __init__(self):
        self.mCellsSize = self.mEdgesSize = self.mMaxEdgesSize = self.mVertexSize = 0
        self.mVertLevels = self.mVertLevelsP1 = 0
        self.mTimesteps = 0
        self.mID = ("", 0)                      # SolutionID {timeStamp, timestep} (MPASOSolution.h:12-16)
        self.mTimeStamp = ""
        self.doubles = {}
        self.cellCenterVelocity = None
        self.cellVertVelocity_vec = None        # [C*(L+1)] vertVelocityTop; None => zero
        self.cellSurfaceHeight = None
        self.mDoubleAttributes = {}

    def init_from_reader(self, reader):
        """MPASOSolution::initSolution(MPASOReader*): raw per-cell arrays, sizes and time stamp."""
        A = AttributeType
        self.mVertLevels, self.mVertLevelsP1 = reader.mVertLevels, reader.mVertLevelsP1
        self.mTimesteps = reader.mTimesteps
        self.mTimeStamp = reader.mTimeStamp
        self.mID = (self.mTimeStamp, self.mTimesteps)   # MPASOSolution.cpp:298-299
        self.doubles = {k: v for k, v in ((A.kLayerThickness, reader.cellLayerThickness_vec),
                                          (A.kBottomDepth, reader.cellBottomDepth_vec),
                                          (A.kZonalVelocity, reader.cellZonalVelocity_vec),
                                          (A.kMeridionalVelocity, reader.cellMeridionalVelocity_vec),
                                          (A.kZTop, reader.cellZTop_vec),
                                          (A.kNormalVelocity, reader.cellNormalVelocity_vec)) if v.size}
        self.cellSurfaceHeight = reader.cellSurfaceHeight_vec if reader.cellSurfaceHeight_vec.size else None
        self.cellVertVelocity_vec = reader.cellVertVelocity_vec if reader.cellVertVelocity_vec.size else None
        for k, v in getattr(reader, "attributes", {}).items():
            self.mDoubleAttributes[k] = v

    def init_from_yaml(self, yaml_path, data_name="", timestep=0):
        self.init_from_reader(MPASOReader.readSolData(yaml_path, data_name, timestep))

    def add_attribute(self, name: str, arr=None):
        """Explicit array, or (pyMOPSAPI: ``add_attribute("temperature", AttributeFormat.kFloat)``) a name the
        reader already loaded; attributes are unobservable in trajectory outputs (Q9)."""
        if arr is not None and not isinstance(arr, (int, enum.Enum)):
            self.mDoubleAttributes[name] = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1)

    def setTimestep(self, t: int):
        self.mTimesteps = int(t)                # like the reference, mID is untouched

    def getID(self) -> int:
        """32-bit FNV-1a of "<timeStamp>_<timestep>" as a signed int (MPASOSolution.h:74-86)."""
        h = 2166136261
        for c in f"{self.mID[0]}_{self.mID[1]}".encode():
            h = ((h ^ c) * 16777619) & 0xFFFFFFFF
        return h - (1 << 32) if h >= (1 << 31) else h

    def getTimeStamp(self) -> str:
        return self.mTimeStamp

    def setAttribute(self, type, val: int):
        name = _GRID_SCALARS.get(GridAttributeType(type))
        if name is None:
            _error("Invalid GridAttributeType")
            return
        setattr(self, name, int(val))

    def setAttributesVec3(self, type, arr):
        if AttributeType(type) != AttributeType.kVelocity:
            _error("Invalid AttributeType")
            return
        self.cellCenterVelocity = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1, 3)

    def setAttributesDouble(self, type, arr):
        self.doubles[AttributeType(type)] = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1)

    def checkAttribute(self) -> bool:
        if AttributeType.kZTop not in self.doubles and AttributeType.kLayerThickness not in self.doubles:
            _error("[MPASOSolution]::Error: Invalid ZTop Attribute")
            return False
        return True


class TrajectorySettings:
    """TrajectorySettings (src/Core/MPASOVisualizer.h:90-103); default method Euler."""

    def __init__(self):
        self.deltaT = 0
        self.simulationDuration = 0
        self.recordT = 0
        self.depth = 0.0
        self.particle_depths = []
        self.fileName = ""
        self.directionType = CalcDirection.kForward
        self.methodType = CalcMethodType.kEuler

    def hasPerParticleDepths(self) -> bool:
        return len(self.particle_depths) > 0


class SeedsSettings:
    """SamplingSettings as bound by pyMOPS (bindings.cpp:225-241)."""

    def __init__(self):
        self._range = (0, 0)
        self._lat = (0.0, 0.0)
        self._lon = (0.0, 0.0)
        self._depth = 0.0

    def setSeedsRange(self, t):
        if len(t) != 2:
            raise RuntimeError("sampleRange must be a tuple of size 2")
        self._range = (int(t[0]), int(t[1]))

    def setGeoBox(self, lat, lon):
        if len(lat) != 2 or len(lon) != 2:
            raise RuntimeError("setGeoBox expects two tuples of size 2")
        self._lat = (float(lat[0]), float(lat[1]))
        self._lon = (float(lon[0]), float(lon[1]))

    def setDepth(self, d: float):
        self._depth = float(d)

    def getDepth(self) -> float:
        return self._depth


# ---- timing (src/Utils/Timer.hpp, categories only) ------------------------

_timing = {"by_category": {}, "records": []}


class _Timer:
    def __init__(self, name, cat):
        self.name, self.cat = name, cat

    def __enter__(self):
        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        ms = (time.perf_counter() - self.t0) * 1e3
        _timing["by_category"][self.cat] = _timing["by_category"].get(self.cat, 0.0) + ms
        _timing["records"].append((self.name, ms))


def MOPS_ResetTiming():
    _timing["by_category"].clear()
    _timing["records"].clear()


def MOPS_PrintTimingSummary():
    print("==== MOPS timing summary (ms) ====")
    for k, v in _timing["by_category"].items():
        print(f"  {k}: {v:.3f}")


def MOPS_PrintTimingDetailed():
    print("==== MOPS timing detailed (ms) ====")
    for k, v in _timing["records"]:
        print(f"  {k}: {v:.3f}")


def MOPS_GetCategoryTime(category: str) -> float:
    return float(_timing["by_category"].get(category, 0.0))


def MOPS_GetTotalTime() -> float:
    return float(sum(_timing["by_category"].values()))


# ---- app state machine (src/Core/MOPS.cpp:10-71, MOPSApp.cpp:34-290) ------

class _App:
    def __init__(self):
        self.configuring = False
        self.grid: MPASOGrid | None = None
        self.sols: dict[int, MPASOSolution] = {}
        self.mesh = None
        self.fields: dict[int, _E.DeviceField] = {}
        self.front = None
        self.back = None


_app = _App()


def MOPS_Init(device: str = "gpu"):
    global _app
    _app = _App()
    _app.grid = MPASOGrid()
    _L.load()  # fail loudly here if the HIP engine is missing


def MOPS_Begin():
    _app.configuring = True


def MOPS_AddGridMesh(grid: MPASOGrid):
    with _Timer("Preprocessing::addGrid", "Preprocessing"):
        _app.grid = grid


def MOPS_AddAttribute(solID: int, sol: MPASOSolution):
    with _Timer("Preprocessing::addSol", "Preprocessing"):
        if solID in _app.sols:  # MOPSApp.cpp:82-87
            return
        g = _app.grid
        sol.mCellsSize, sol.mEdgesSize, sol.mMaxEdgesSize, sol.mVertexSize = \
            g.mCellsSize, g.mEdgesSize, g.mMaxEdgesSize, g.mVertexSize
        g.mVertLevels, g.mVertLevelsP1 = sol.mVertLevels, sol.mVertLevelsP1
        _app.sols[solID] = sol


def MOPS_End():
    if not _app.configuring:  # MOPS.cpp:31-46
        print(" [ MOPS is not configuring ]", file=sys.stderr)
        sys.exit(1)
    ok = _app.grid is not None and bool(_app.grid.checkAttribute())
    ok = ok and all(s.checkAttribute() for s in _app.sols.values())
    if not ok:
        print(" [ MOPS is not configured ]", file=sys.stderr)
        sys.exit(1)
    _app.configuring = False
    with _Timer("Preprocessing::upload", "Preprocessing"):
        g = _app.grid
        G = GridAttributeType
        _app.mesh = _E.DeviceMesh(nCells=g.mCellsSize, nVertices=g.mVertexSize, maxEdges=g.mMaxEdgesSize,
                                  nVertLevels=g.mVertLevels, nEdgesOnCell=g.ints[G.kNumberVertexOnCell],
                                  verticesOnCell=g.ints[G.kVerticesOnCell], cellsOnCell=g.ints[G.kCellsOnCell],
                                  cellsOnVertex=g.ints[G.kCellsOnVertex], cellCoord=g.vec3[G.kCellCoord],
                                  vertexCoord=g.vec3[G.kVertexCoord])
        A = AttributeType
        # a solution with the edge-normal velocity only (kNormalVelocity) takes the RBF reconstruction
        # (MPASOSolution::calcCellCenterVelocity), which needs the grid's edges on the device
        rbf = {sid: (s.doubles.get(A.kZonalVelocity) is None or s.doubles.get(A.kMeridionalVelocity) is None)
               and s.doubles.get(A.kNormalVelocity) is not None for sid, s in _app.sols.items()}
        if any(rbf.values()):
            _app.mesh.set_edges(len(g.vec3[G.kEdgeCoord]), g.ints[G.kEdgesOnCell], g.ints[G.kCellsOnEdge],
                                g.vec3[G.kEdgeCoord])
        for sid, s in sorted(_app.sols.items()):
            snap = types.SimpleNamespace(
                timestep=s.mTimesteps, layerThickness=s.doubles.get(A.kLayerThickness),
                bottomDepth=s.doubles.get(A.kBottomDepth), surfaceHeight=s.cellSurfaceHeight,
                zonalVelocity=s.doubles.get(A.kZonalVelocity),
                meridionalVelocity=s.doubles.get(A.kMeridionalVelocity), vertVelocityTop=s.cellVertVelocity_vec,
                normalVelocity=s.doubles.get(A.kNormalVelocity))
            _app.fields[sid] = _E.DeviceField.from_snapshot(_app.mesh, snap,
                                                            velocity="rbf" if rbf[sid] else "zonal")
        if _app.fields:
            _app.front = _app.fields[min(_app.fields)]


def MOPS_ActiveAttribute(t1: int, t2: int | None = None):
    _app.front = _app.back = None
    if t1 not in _app.fields or (t2 is not None and t2 not in _app.fields):
        _error(f"[MOPSApp]::activeAttribute: solID {t1 if t1 not in _app.fields else t2} not found")
        return
    _app.front = _app.fields[t1]
    _app.back = None if t2 is None else _app.fields[t2]


def MOPS_GenerateSeedsPoints(setting: SeedsSettings) -> np.ndarray:
    """MPASOVisualizer::GenerateSamplePoint (MPASOVisualizer.cpp:120-149): exclusive upper bounds."""
    (min_lat, max_lat), (min_lon, max_lon) = setting._lat, setting._lon
    i_step = (max_lat - min_lat) / float(setting._range[0] - 1)
    j_step = (max_lon - min_lon) / float(setting._range[1] - 1)
    pts = []
    i = min_lat
    while i < max_lat:
        j = min_lon
        while j < max_lon:
            pts.append((j, i))
            j += j_step
        i += i_step
    r = float(np.float32(6371010.0))
    out = np.empty((len(pts), 3))
    for k, (lon_d, lat_d) in enumerate(pts):
        lat, lon = lat_d * (math.pi / 180.0), lon_d * (math.pi / 180.0)
        ct, cp, st, sp = math.cos(lat), math.cos(lon), math.sin(lat), math.sin(lon)
        out[k] = (r * ct * cp, r * ct * sp, r * st)
    return out


def _run(config: TrajectorySettings, sample_points_np, pathline: bool, stage: str):
    a = np.asarray(sample_points_np)
    if a.ndim != 2 or a.shape[1] != 3:
        raise RuntimeError("Input sample_points must be a (N, 3) numpy array.")
    seeds = np.ascontiguousarray(a, dtype=np.float64)
    if config is None or _app.front is None or (pathline and _app.back is None):
        _error(f"[{stage}] invalid inputs")
        return None, seeds, None
    if len(seeds) == 0:
        return None, seeds, None
    if config.deltaT == 0 or config.recordT == 0 or config.simulationDuration == 0:
        _error(f"[{stage}] invalid trajectory settings")
        return None, seeds, None
    depths = None
    if config.hasPerParticleDepths() and len(config.particle_depths) == len(seeds):
        depths = np.asarray(config.particle_depths, dtype=np.float32)
    eff = depths if depths is not None else np.full(len(seeds), np.float32(config.depth), dtype=np.float32)
    cfg = _E.TrajectoryConfig(deltaT=int(config.deltaT), simulationDuration=int(config.simulationDuration),
                              recordT=int(config.recordT), depth=float(np.float32(config.depth)),
                              direction=int(config.directionType), method=int(config.methodType))
    if cfg.n_records <= 0 or cfg.n_steps <= 0:
        _error(f"[{stage}] invalid integration steps")  # seed-only lines (:709-712)
        return "seed_only", seeds, eff
    r = _E.run_trajectories(_app.mesh, _app.front, _app.back if pathline else None, cfg, seeds, depths=depths)
    return r, seeds, eff


def MOPS_RunStreamLine(config: TrajectorySettings, sample_points_np):
    with _Timer("GPUKernel::StreamLine", "GPUKernel"):
        r, seeds, _ = _run(config, sample_points_np, False, "MI355X::StreamLine")
        if r is None:
            return []
        if isinstance(r, str):  # velocity shorter than points -> NaN rows (bindings.cpp:356-360)
            return [{"lineID": i, "points": seeds[i:i + 1].copy(), "velocity": np.full((1, 3), np.nan)}
                    for i in range(len(seeds))]
        return [{"lineID": i, "points": r["points"][i], "velocity": r["velocity"][i]} for i in range(len(seeds))]


def MOPS_RunPathLine(config: TrajectorySettings, sample_points_np):
    with _Timer("GPUKernel::PathLine", "GPUKernel"):
        if _app.front is None or _app.back is None:  # MOPSApp.cpp:259-271
            _error("[MOPSApp]::Sol_Front or Sol_Back is nullptr, please activeAttribute first")
            sys.exit(-1)
        r, seeds, eff = _run(config, sample_points_np, True, "MI355X::PathLine")
        if r is None:
            return []
        if isinstance(r, str):
            return [{"lineID": i, "points": seeds[i:i + 1].copy(), "velocity": np.zeros((1, 3)),
                     "temperature": np.zeros(1), "salinity": np.zeros(1), "lastPoint": seeds[i].copy(),
                     "depth": float(eff[i])} for i in range(len(seeds))]
        return [{"lineID": i, "points": r["points"][i], "velocity": r["velocity"][i],
                 "temperature": r["temperature"][i], "salinity": r["salinity"][i], "lastPoint": r["lastPoint"][i],
                 "depth": float(eff[i])} for i in range(len(seeds))]


def MOPS_RunRemapping(config):
    raise NotImplementedError("image remapping is out of scope for the trajectory engine (DESIGN.md)")


def MOPS_RunReGrid(config):
    raise NotImplementedError("regridding is out of scope for the trajectory engine (DESIGN.md)")
