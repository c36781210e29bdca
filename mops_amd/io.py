"""Trajectory output formats (include/mops_io.h), Python side.

``lines`` is the dict the engine returns (``run_trajectories``,
``ParticleSet.finalize``, ``PathlineChain.run``): points/velocity [n, P, 3],
temperature/salinity [n, P], as numpy arrays or device tensors.  The
xyz -> (lat, lon, r, |v|) conversion runs on the GPU (``lines_geo``); the
writers stream to disk in native code.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def _host(a):
    if a is None:
        return None
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def lines_geo(points, velocity=None, stream=None):
    """Device {lat_deg, lon_deg, r, |v|} per point (mops_lines_geo) -> torch [n, P, 4]."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    p = torch.as_tensor(points, dtype=torch.float64, device=dev).contiguous()
    v = None if velocity is None else torch.as_tensor(velocity, dtype=torch.float64, device=dev).contiguous()
    n, P = int(p.shape[0]), int(p.shape[1])
    out = torch.empty((n, P, 4), dtype=torch.float64, device=dev)
    h = C.c_void_p(0 if stream is None else int(getattr(stream, "cuda_stream", stream)))
    L.check(L.load().mops_lines_geo(n, P, C.c_void_p(p.data_ptr()), None if v is None else C.c_void_p(v.data_ptr()),
                                    C.c_void_p(out.data_ptr()), h), "mops_lines_geo")
    return out


def save_trajectory_lines_vtp(path: str, lines: dict, binary: bool = True, geo=None):
    """VTKFileManager::SaveTrajectoryLinesAsVTP (VTKFileManager.hpp:315-417)."""
    pts = lines["points"]
    n, P = int(pts.shape[0]), int(pts.shape[1])
    g = _host(geo if geo is not None else lines_geo(pts, lines.get("velocity")))
    t, s = _host(lines.get("temperature")), _host(lines.get("salinity"))
    L.check(L.load().mops_write_lines_vtp(path.encode(), n, P, _ptr(g), _ptr(t), _ptr(s), 1 if binary else 0),
            "mops_write_lines_vtp")


def save_trajectory_lines_txt(path: str, lines: dict):
    """The CLI's text dump (CLI/main.cpp:239-262)."""
    p, v = _host(lines["points"]), _host(lines["velocity"])
    L.check(L.load().mops_write_lines_txt(path.encode(), p.shape[0], p.shape[1], _ptr(p), _ptr(v)),
            "mops_write_lines_txt")


def export_pathlines_to_binary(lines: dict, path: str, include_velocity: bool = False,
                               include_scalars: bool = False, geo=None):
    """tutorial/export_pathline_binary.py:export_pathlines_to_binary (+ .meta.json)."""
    pts = lines["points"]
    n, P = int(pts.shape[0]), int(pts.shape[1])
    g = _host(geo if geo is not None else lines_geo(pts, lines.get("velocity")))
    v = _host(lines.get("velocity")) if include_velocity else None
    t = _host(lines.get("temperature")) if include_scalars else None
    s = _host(lines.get("salinity")) if include_scalars else None
    L.check(L.load().mops_write_pathline_binary(path.encode(), n, P, _ptr(g), _ptr(v), _ptr(t), _ptr(s),
                                                int(include_velocity), int(include_scalars)),
            "mops_write_pathline_binary")
