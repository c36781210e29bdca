"""MOPS_CLI mirror (mops_amd/cli.py over CLI/main.cpp).

CPU: the cxxopts surface (options, defaults, comma lists, the required input).
GPU: a whole CLI run on a small MPAS-layout netCDF dataset (the fixtures of
test_mpas_reader.py) -- its text dump must equal the one written from the
oracle's lines for the same lattice, settings and snapshot, character for
character.
"""
import os

import numpy as np
import pytest


def test_cli_options():
    from mops_amd.cli import parse_command_line
    a = parse_command_line(["-i", "x.yaml"])
    assert (a.input, a.prefix, a.timestep, a.range, a.day, a.depth) == ("x.yaml", "", 0, [], 1, 10.0)
    a = parse_command_line(["--input", "y.yaml", "-p", "/d", "-t", "3", "-r", "1,2", "-r", "5", "-g", "2", "-d", "800"])
    assert (a.input, a.prefix, a.timestep, a.range, a.day, a.depth) == ("y.yaml", "/d", 3, [1, 2, 5], 2, 800.0)
    assert parse_command_line([]) is None            # "[ERROR]::Input yaml file is required."
    assert parse_command_line(["-h", "-i", "x"]) is None


@pytest.mark.gpu
def test_cli_streamline_matches_oracle(engine_lib, oracle_lib, gpu, tmp_path, monkeypatch):
    from test_mpas_reader import YAML, _mesh, _write_hist, _write_mesh
    from mops_amd import cli, io as mio, pyMOPS as M
    mesh, snaps = _mesh()
    _write_mesh(str(tmp_path / "mesh.nc"), mesh, 2)
    _write_hist(str(tmp_path / "hist.am.timeSeriesStatsMonthly.0001-01-01.nc"), mesh, snaps[:2], 2, 1)
    y = tmp_path / "mpas.yaml"
    y.write_text(YAML.format(prefix=str(tmp_path)))
    monkeypatch.chdir(tmp_path)
    assert cli.main(["-i", str(y), "-t", "1", "-d", "150", "-g", "1"]) == 0
    got = (tmp_path / "traj_line_1.txt").read_text()
    assert (tmp_path / "traj_line_1.vtp").stat().st_size > 0
    # the same run through the oracle: lattice, snapshot 1, dt 1 h, 1 day, record 6 h, depth 150 m
    ss = M.SeedsSettings(); ss.setSeedsRange((31, 31)); ss.setGeoBox((35.0, 45.0), (-90.0, -15.0))
    seeds = M.MOPS_GenerateSeedsPoints(ss)
    ref = oracle_lib.run(mesh, oracle_lib.preprocess(mesh, snaps[1]), None, seeds, depth=150.0, delta_t=3600,
                         duration=86400, record_t=6 * 3600, euler=True)
    mio.save_trajectory_lines_txt(str(tmp_path / "ref.txt"), {"points": ref["points"], "velocity": ref["velocity"]})
    assert got == (tmp_path / "ref.txt").read_text()
