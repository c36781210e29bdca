"""MOPSPathline (mops_amd/pathline.py), the tutorial's month-pair caller (tutorial/pyMOPSAPI.py:1179-1531),
end to end: MPAS-format monthly history files with xtime_startMonthly stamps are read through the YAML
stream, the chain runs January (31 days) and February (28 days) with each pair's duration from the
stamps, and the concatenated lines equal the oracle chain run with the same gaps bit for bit; a second
run() continues the same particles from their last points, as the reference's stateful class does."""
import importlib.util
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
scipy_io = pytest.importorskip("scipy.io")

HERE = os.path.dirname(os.path.abspath(__file__))


def _module(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(HERE, name + ".py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _write_month(path, mesh, snap, stamp):
    C, L = mesh.nCells, mesh.nVertLevels
    f = scipy_io.netcdf_file(path, "w", version=2)
    f.createDimension("Time", None); f.createDimension("nCells", C)
    f.createDimension("nVertLevels", L); f.createDimension("nVertLevelsP1", L + 1); f.createDimension("StrLen", 64)
    xt = f.createVariable("xtime_startMonthly", "c", ("Time", "StrLen"))
    lt = f.createVariable("timeMonthly_avg_layerThickness", "d", ("Time", "nCells", "nVertLevels"))
    vz = f.createVariable("timeMonthly_avg_velocityZonal", "d", ("Time", "nCells", "nVertLevels"))
    vm = f.createVariable("timeMonthly_avg_velocityMeridional", "d", ("Time", "nCells", "nVertLevels"))
    vv = f.createVariable("timeMonthly_avg_vertVelocityTop", "d", ("Time", "nCells", "nVertLevelsP1"))
    f.createVariable("bottomDepth", "d", ("nCells",))[:] = snap.bottomDepth
    xt[0] = np.frombuffer(stamp.ljust(64, "\0").encode(), dtype="S1")
    lt[0] = snap.layerThickness.reshape(C, L)
    vz[0] = snap.zonalVelocity.reshape(C, L)
    vm[0] = snap.meridionalVelocity.reshape(C, L)
    vv[0] = snap.vertVelocityTop.reshape(C, L + 1)
    f.close()


def test_mopspathline_month_pairs_match_oracle(engine_lib, oracle_lib, gpu, tmp_path):
    from mops_amd import synth
    from mops_amd.pathline import MOPSPathline
    rd = _module("test_mpas_reader")
    oracle_chain = _module("test_chain").oracle_chain
    mesh = synth.make_mesh(8, n_levels=6)
    snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.3 * t) for t in range(4)]
    rd._write_mesh(str(tmp_path / "mesh.nc"), mesh, 2)
    dates = ["0001-01-01", "0001-02-01", "0001-03-01", "0001-04-01"]
    for d, s in zip(dates, snaps):
        _write_month(str(tmp_path / f"hist.am.timeSeriesStatsMonthly.{d}.nc"), mesh, s, d + "_00:00:00")
    y = tmp_path / "mpas.yaml"
    y.write_text(rd.YAML.format(prefix=str(tmp_path)))
    seeds = synth.uniform_band_seeds(90, seed=4)

    p = MOPSPathline(str(y)).init("gpu")
    p.set_time(1, 1, 1, 3)
    assert p.pairs == [("0001-01-01", "0001-02-01"), ("0001-02-01", "0001-03-01")]
    p.set_seed(depth=150.0, points=seeds)
    lines = p.run(method="euler", delta_minutes=180, record_every_minutes=1440)
    gaps = [31 * 86400, 28 * 86400]
    ref = oracle_chain(oracle_lib, mesh, snaps[:3], seeds, 150.0, None, gaps, 10800, 86400, euler=True)
    assert len(lines) == len(seeds) and lines[0]["points"].shape == (1 + 31 + 28, 3)
    for k in ("points", "velocity", "temperature", "salinity", "lastPoint"):
        got = np.stack([ln[k] for ln in lines])
        assert np.array_equal(got, ref[k]), k
    assert [ln["lineID"] for ln in lines] == list(range(len(seeds)))

    # the stateful continuation: March from the particles' last points (_first_round False)
    p.set_time(1, 3, 1, 4)
    lines2 = p.run(method="euler", delta_minutes=180, record_every_minutes=1440)
    ref2 = oracle_chain(oracle_lib, mesh, snaps[2:4], ref["lastPoint"], 150.0, None, [31 * 86400], 10800, 86400,
                        euler=True)
    assert np.array_equal(np.stack([ln["points"] for ln in lines2]), ref2["points"])
    # reset_segments: back to the configured seeds
    p.reset_segments()
    p.set_time(1, 1, 1, 2)
    lines3 = p.run(method="euler", delta_minutes=180, record_every_minutes=1440)
    assert np.array_equal(np.stack([ln["points"] for ln in lines3]), ref["points"][:, :32])
