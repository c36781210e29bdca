"""Golden vectors for the pathline binary export (tests/test_io_golden.py).

Runs the reference's own exporter, ``export_pathlines_to_binary`` from
/root/reference/tutorial/export_pathline_binary.py (pure numpy + struct +
json), on fixed synthetic pathlines and commits its outputs as fixtures:

  pathline_binary_inputs.npz          the lines (points, velocity, temperature, salinity)
  pathline_binary_<tag>.bin / .meta.json   for (include_velocity, include_scalars) per tag

Only this generator imports the reference, and only in the build container
(the GPU box has no /root/reference): ``python tests/golden/make_pathline_binary.py``.
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/tutorial/export_pathline_binary.py"
TAGS = {"plain": (False, False), "vel": (True, False), "vel_scalars": (True, True)}


def make_lines():
    """6 pathlines x 9 points on shells around 6.371e6 m: mid-latitudes, both poles' vicinity,
    the dateline crossed both ways, the prime meridian and the equator."""
    rng = np.random.default_rng(20261017)
    lat0 = np.radians([35.0, -62.5, 89.2, -88.7, 0.0, 12.25])
    lon0 = np.radians([-170.0, 179.5, 45.0, -120.0, 0.0, -179.9])
    dlon = np.radians([-2.0, 1.5, 30.0, -25.0, 0.7, -0.05])
    P = 9
    lines = []
    for i in range(len(lat0)):
        k = np.arange(P)
        lat = lat0[i] + np.radians(0.05) * np.sin(k + i)
        lon = lon0[i] + dlon[i] * k / (P - 1)
        r = 6_371_000.0 - rng.uniform(0.0, 2500.0, P)  # depths of up to 2.5 km
        pts = np.stack([r * np.cos(lat) * np.cos(lon), r * np.cos(lat) * np.sin(lon), r * np.sin(lat)], axis=1)
        vel = rng.normal(scale=0.3, size=(P, 3))
        vel[-1] = 0.0  # the zero the reference appends to every line's velocity
        tmp = rng.uniform(-2.0, 30.0, P)
        sal = rng.uniform(30.0, 38.0, P)
        lines.append(dict(points=pts, velocity=vel, temperature=tmp, salinity=sal))
    return lines


def main():
    spec = importlib.util.spec_from_file_location("export_pathline_binary", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    lines = make_lines()
    np.savez(os.path.join(HERE, "pathline_binary_inputs.npz"),
             points=np.stack([l["points"] for l in lines]), velocity=np.stack([l["velocity"] for l in lines]),
             temperature=np.stack([l["temperature"] for l in lines]),
             salinity=np.stack([l["salinity"] for l in lines]))
    for tag, (vel, sca) in TAGS.items():
        mod.export_pathlines_to_binary(lines, os.path.join(HERE, f"pathline_binary_{tag}.bin"), include_velocity=vel,
                                       include_scalars=sca)
    print("numpy", np.__version__, file=sys.stderr)


if __name__ == "__main__":
    main()
