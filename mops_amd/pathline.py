"""MOPSPathline: the reference's month-pair pathline caller on the device-resident chain.

Mirrors ``MOPSPathline`` of tutorial/pyMOPSAPI.py:1179-1531 -- the same methods, argument meaning,
state and result layout -- so a script written against the tutorial class runs unchanged:

    p = MOPSPathline("mpas.yaml").init("gpu")
    p.set_time(1, 1, 2, 1, direction="forward")          # month pairs (_month_pairs_forward)
    p.set_seed(depth=20.0, lat_range=(18, 31), lon_range=(-98, -80), grid=(40, 40))
    lines = p.run(method="rk4", delta_minutes=1, record_every_minutes=6)

The reference re-registers the grid and both solutions with MOPS and runs one PathLine per pair,
preprocessing every snapshot on the host each time.  Here the whole schedule is one
``chain.PathlineChain`` run: the grid is uploaded once, each snapshot read once (MPASOReader) and
derived on the device, continuation points, per-particle depths and lines stay in HBM, and each pair's
simulationDuration comes from the snapshots' xtime (``_time_gap_seconds``, :1444) -- read ahead with
``MPASOReader.readTimeStamp`` so that every pair's step and record counts are known up front.

State across run() calls is the reference's: after a run, the next run continues the same particles
from their last points (``_first_round`` / ``_last_pt``) until ``reset_segments``.
"""
from __future__ import annotations

import numpy as np

from . import chain as _chain
from . import _lib as L

EARTH_RADIUS_M = _chain.EARTH_RADIUS_M  # pyMOPSAPI.py:46


class MOPSPathline:
    def __init__(self, yaml_path: str):
        self.yaml_path = yaml_path
        self.pairs = None
        self.direction = "forward"
        self._seed_conf = None
        self._seed_points = None
        self._follow_last = True
        self._first_round = True
        self._depth = None
        self._particle_depths = None
        self._last_pt = None
        self._one_min = 60
        self._grid = None
        self._mesh = None   # DeviceMesh, built at the first run (its level count comes from a solution)
        self.device = None

    # ---- MOPSPathline static helpers (pyMOPSAPI.py:1235-1295)
    _month_pairs_forward = staticmethod(_chain.month_pairs_forward)
    _month_pairs_backward = staticmethod(_chain.month_pairs_backward)
    _time_gap_seconds = staticmethod(_chain.time_gap_seconds)

    @staticmethod
    def _to_int_ymd(s: str) -> int:  # "0018-01-01" -> 180101 (pyMOPSAPI.py:1281-1283)
        y, mo, d = s.split("-")
        return int(y) * 10000 + int(mo) * 100 + int(d)

    def reset_segments(self):
        """The next run() starts a new sequence from the configured seeds (pyMOPSAPI.py:1219-1233)."""
        self._first_round = True
        self._last_pt = None

    def init(self, device: str = "gpu"):
        """Load the static grid (pyMOPSAPI.py:1300-1305).  ``device`` is accepted for the reference's
        signature; the engine runs on the current HIP device."""
        import torch
        from .mpas import MPASOReader
        if device not in ("gpu", "cpu", "cuda"):
            raise ValueError(f"unknown device {device!r}")
        self.device = torch.device("cuda", torch.cuda.current_device())
        self._grid = MPASOReader.readGridData(self.yaml_path)
        self._mesh = None
        return self

    def set_time(self, sy: int, sm: int, ey: int, em: int, direction: str = "forward"):
        """Month pairs and direction (pyMOPSAPI.py:1310-1327)."""
        self.direction = direction.lower()
        if self.direction == "forward":
            self.pairs = self._month_pairs_forward(sy, sm, ey, em)
        elif self.direction == "backward":
            self.pairs = self._month_pairs_backward(sy, sm, ey, em)
        else:
            raise ValueError("direction must be 'forward' or 'backward'")
        if not self.pairs:
            raise ValueError("no month pairs produced; check input range")
        return self

    def set_seed(self, depth: float = None, depths=None, lat_range: tuple = None, lon_range: tuple = None,
                 grid: tuple = (2, 2), points=None, follow_last: bool = True):
        """Seeds: explicit (N, 3) points with an optional per-particle depth each, or a lat/lon lattice
        at one depth (pyMOPSAPI.py:1332-1391)."""
        from . import pyMOPS
        self._follow_last = bool(follow_last)
        if depths is not None:
            self._particle_depths = np.asarray(depths, dtype=np.float32).flatten()
            self._depth = float(self._particle_depths[0])
        elif depth is not None:
            self._depth = float(depth)
            self._particle_depths = None
        else:
            raise ValueError("must provide either 'depth' (scalar) or 'depths' (array)")
        if points is not None:
            arr = np.asarray(points, dtype=float)
            if arr.ndim != 2 or arr.shape[1] != 3:
                raise ValueError("points must be a (N,3) array")
            self._seed_points = arr.copy()
            self._seed_conf = None
            if self._particle_depths is not None and len(self._particle_depths) != arr.shape[0]:
                raise ValueError(f"depths length ({len(self._particle_depths)}) must match points count "
                                 f"({arr.shape[0]})")
        else:
            if not (lat_range and lon_range):
                raise ValueError("when points is None, must provide lat_range & lon_range")
            if self._particle_depths is not None:
                raise ValueError("per-particle depths only supported when providing explicit points")
            nx, ny = grid
            conf = pyMOPS.SeedsSettings()
            conf.setSeedsRange((int(nx), int(ny)))
            conf.setGeoBox(tuple(map(float, lat_range)), tuple(map(float, lon_range)))
            conf.setDepth(self._depth)
            self._seed_conf = conf
            self._seed_points = None
        return self

    def _seeds(self):
        from . import pyMOPS
        if self._first_round or not self._follow_last:
            if self._seed_points is not None:
                return self._seed_points.copy()
            return pyMOPS.MOPS_GenerateSeedsPoints(self._seed_conf)
        if self._last_pt is None:
            raise RuntimeError("follow_last=True but last_pts is None")
        return self._last_pt.copy()

    def run(self, method: str = "rk4", delta_minutes: int = 1, record_every_minutes: int = 6) -> list:
        """All month pairs as one device-resident chain; the per-pair lines concatenated (later pairs
        without their first sample), pyMOPSAPI.py:1396-1531.  Returns list[dict] with lineID, points
        (M, 3), velocity (M, 3), temperature (M,), salinity (M,), lastPoint (3,)."""
        from .chain import PathlineChain
        from .engine import DeviceField, DeviceMesh
        from .mpas import MPASOReader, mesh_from_reader, snapshot_from_reader
        if self.pairs is None:
            raise RuntimeError("call set_time(...) before run()")
        if self._depth is None:
            raise RuntimeError("call set_seed(...) before run()")
        if self._grid is None:
            raise RuntimeError("call init(...) before run()")
        dates = [a for a, _ in self.pairs] + [self.pairs[-1][1]]
        stamps = [MPASOReader.readTimeStamp(self.yaml_path, d, 0) for d in dates]
        if self._mesh is None:
            first = MPASOReader.readSolData(self.yaml_path, dates[0], 0)
            self._mesh = DeviceMesh.from_mesh(mesh_from_reader(self._grid, first.mVertLevels))

        def make_field(i, stream):  # snapshot i read from its file and derived on the device
            sol = MPASOReader.readSolData(self.yaml_path, dates[i], 0)
            return DeviceField.from_snapshot(self._mesh, snapshot_from_reader(sol, timestep_id=i), stream=stream)

        seeds = self._seeds()
        pdep = None
        if self._particle_depths is not None:
            pdep = self._particle_depths
            if self._follow_last and not self._first_round:  # :1465-1469
                pdep = np.clip(EARTH_RADIUS_M - np.linalg.norm(seeds, axis=1), 0.0, None).astype(np.float32)
        chain = PathlineChain(self._mesh, make_field, len(dates), timestamps=stamps, device=self.device)
        res = chain.run(seeds, depth=self._depth, particle_depths=pdep,
                        method=L.MOPS_RK4 if method.lower() == "rk4" else L.MOPS_EULER,
                        delta_t=int(delta_minutes) * self._one_min,
                        record_t=int(record_every_minutes) * self._one_min,
                        direction=L.MOPS_FORWARD if self.direction == "forward" else L.MOPS_BACKWARD,
                        follow_last=self._follow_last)
        out = {k: res[k].cpu().numpy() for k in ("points", "velocity", "temperature", "salinity", "lastPoint")}
        self._last_pt = out["lastPoint"].astype(float, copy=True)
        if self._particle_depths is not None:  # :1491-1495
            self._particle_depths = np.clip(EARTH_RADIUS_M - np.linalg.norm(self._last_pt, axis=1), 0.0,
                                            None).astype(np.float32)
        self._first_round = False
        return [dict(lineID=i, points=out["points"][i], velocity=out["velocity"][i],
                     temperature=out["temperature"][i], salinity=out["salinity"][i], lastPoint=out["lastPoint"][i])
                for i in range(out["points"].shape[0])]
