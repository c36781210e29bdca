"""Diagnostic for tests/test_pathline_api.py: where do MOPSPathline's lines and the oracle chain part?"""
import importlib.util
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _module(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tests", name + ".py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    from mops_amd import synth
    from mops_amd.chain import PathlineChain, snapshot_field_factory
    from mops_amd.engine import DeviceMesh
    from mops_amd.mpas import MPASOReader, mesh_from_reader, snapshot_from_reader
    from mops_amd.pathline import MOPSPathline
    from oracle import oracle as O
    O.build()
    rd = _module("test_mpas_reader")
    api = _module("test_pathline_api")
    oracle_chain = _module("test_chain").oracle_chain
    tmp = tempfile.mkdtemp()
    mesh = synth.make_mesh(8, n_levels=6)
    snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.3 * t) for t in range(3)]
    rd._write_mesh(os.path.join(tmp, "mesh.nc"), mesh, 2)
    dates = ["0001-01-01", "0001-02-01", "0001-03-01"]
    for d, s in zip(dates, snaps):
        api._write_month(os.path.join(tmp, f"hist.am.timeSeriesStatsMonthly.{d}.nc"), mesh, s, d + "_00:00:00")
    y = os.path.join(tmp, "mpas.yaml")
    open(y, "w").write(rd.YAML.format(prefix=tmp))
    seeds = synth.uniform_band_seeds(90, seed=4)
    gaps = [31 * 86400, 28 * 86400]
    ref = oracle_chain(O, mesh, snaps, seeds, 150.0, None, gaps, 10800, 86400, euler=True)
    # 1. the API
    p = MOPSPathline(y).init("gpu").set_time(1, 1, 1, 3).set_seed(depth=150.0, points=seeds)
    lines = p.run(method="euler", delta_minutes=180, record_every_minutes=1440)
    got = np.stack([ln["points"] for ln in lines])
    # 2. the chain on the synthetic snapshots
    dm = DeviceMesh.from_mesh(mesh)
    ch = PathlineChain(dm, snapshot_field_factory(dm, lambda i: snaps[i]), 3, gap_seconds=gaps)
    got2 = ch.run(seeds, depth=150.0, method=1, delta_t=10800, record_t=86400)["points"].cpu().numpy()
    # 3. the chain on the reader's snapshots
    rsn = [snapshot_from_reader(MPASOReader.readSolData(y, d, 0), timestep_id=i) for i, d in enumerate(dates)]
    g = MPASOReader.readGridData(y)
    dm3 = DeviceMesh.from_mesh(mesh_from_reader(g, 6))
    ch3 = PathlineChain(dm3, snapshot_field_factory(dm3, lambda i: rsn[i]), 3, gap_seconds=gaps)
    got3 = ch3.run(seeds, depth=150.0, method=1, delta_t=10800, record_t=86400)["points"].cpu().numpy()
    for name, a in (("api", got), ("chain synth", got2), ("chain reader", got3)):
        eq = np.all(a == ref["points"], axis=-1)
        bad = np.argwhere(~eq)
        print(name, "equal lines", int(np.all(eq, axis=1).sum()), "of", a.shape[0], "first bad (line, point)",
              bad[:3].tolist(), "nan", int(np.isnan(a).sum()), int(np.isnan(ref["points"]).sum()))
        if len(bad):
            i, j = bad[0]
            print("   got", a[i, j], "ref", ref["points"][i, j])
    for k in ("bottomDepth", "layerThickness", "zonalVelocity", "meridionalVelocity", "vertVelocityTop"):
        print(k, all(np.array_equal(getattr(rsn[t], k), getattr(snaps[t], k)) for t in range(3)))
    print("surfaceHeight synth", getattr(snaps[0], "surfaceHeight", None) is not None, "reader", rsn[0].surfaceHeight)


if __name__ == "__main__":
    main()
