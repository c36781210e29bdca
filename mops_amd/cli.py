"""MOPS_CLI on the MI355X engine: ``python -m mops_amd.cli -i <yaml> [...]``.

Mirrors the reference's command-line driver (CLI/main.cpp) option for option:

    -i/--input     ftk stream YAML (required)          cxxopts "input,i"
    -p/--prefix    data path prefix                     "prefix,p"
    -t/--timestep  single timestep (default 0)          "timestep,t"
    -r/--range     timestep list ("-r 1,2" or repeated) "range,r"
    -g/--day       day gap (default 1)                  "day,g"
    -d/--depth     fixed depth in metres (default 10)   "depth,d"

and its run (CLI/main.cpp:94-262): grid and one solution per timestep from the
YAML (initGrid_DemoLoading / initSolution_DemoLoading, with temperature and
salinity attributes), a 31x31 sample lattice in lat [35, 45), lon [-90, -15)
at the fixed depth, and -- for a single timestep -- a StreamLine with
deltaT = 1 h, simulationDuration = day_gap days, recordT = 6 h, written as
``traj_line_<t>.txt`` (the reference's text dump) and ``traj_line_<t>.vtp``
(its VTK build's SaveTrajectoryLinesAsVTP) in the working directory.

The per-timestep remapping images (MOPS_RunRemapping, PNG/VTI) are out of scope
of this build; the CLI says so and goes on, as the reference
does when a stage produces nothing.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

ONE_HOUR = 3600
ONE_DAY = 86400


def _int_list(values):
    out = []
    for v in values or []:
        out.extend(int(x) for x in str(v).split(",") if x.strip())
    return out


def parse_command_line(argv):
    """CLI/main.cpp:28-56 (cxxopts); returns None where the reference returns false (help, no input)."""
    p = argparse.ArgumentParser(prog="MOPS_CLI", add_help=False)
    p.add_argument("-i", "--input", default=None, help="Input yaml file")
    p.add_argument("-p", "--prefix", default="", help="Data path prefix")
    p.add_argument("-t", "--timestep", type=int, default=0, help="single timestep")
    p.add_argument("-r", "--range", action="append", default=None, help="Timestep range")
    p.add_argument("-g", "--day", type=int, default=1, help="Day Gap")
    p.add_argument("-d", "--depth", type=float, default=10.0, help="Fixed depth")
    p.add_argument("-h", "--help", action="store_true", help="Print this information")
    args = p.parse_args(argv)
    if args.help:
        print(p.format_help())
        return None
    if not args.input:
        print("[ERROR]::Input yaml file is required.")
        return None
    args.range = _int_list(args.range)
    return args


def main(argv=None) -> int:
    args = parse_command_line(sys.argv[1:] if argv is None else argv)
    if args is None:
        return 1
    print("== command line arguments ==")
    print(f"== input_yaml_filename: {args.input}")
    print(f"== data_path_prefix: {args.prefix}")
    print(f"== timestep: {args.timestep}")
    print(f"== day_gap: {args.day}")
    print(f"== fixed_depth: {args.depth}")
    print("== time_range_vec: " + "".join(f"{t} " for t in args.range))

    from . import io as mio
    from . import pyMOPS as M

    # 1-4. engine, grid, one solution per timestep, attributes
    M.MOPS_Init("gpu")
    timesteps = list(args.range) if args.range else [args.timestep]
    grid = M.MPASOGrid()
    grid.init_from_yaml(args.input)
    sols = []
    for t in timesteps:
        s = M.MPASOSolution()
        s.init_from_yaml(args.input, "", t)       # initSolution_DemoLoading(yaml, t)
        s.add_attribute("temperature")
        s.add_attribute("salinity")
        sols.append(s)
    M.MOPS_Begin()
    M.MOPS_AddGridMesh(grid)
    for t, s in zip(timesteps, sols):
        M.MOPS_AddAttribute(t, s)
    M.MOPS_End()

    # 5-6. per-timestep remapping (out of scope); the last timestep stays active, as in the reference
    for t in timesteps:
        M.MOPS_ActiveAttribute(t)
        print(f"[MOPS_CLI] timestep {t}: remapping images (MOPS_RunRemapping) are not part of this build; skipped")

    # 7. sample points: 31 x 31 lattice request in [35, 45] x [-90, -15] (exclusive upper bounds)
    print("== generate sample points ==")
    ss = M.SeedsSettings()                    # SamplingSettings, atCellCenter(false)
    ss.setSeedsRange((31, 31))
    ss.setGeoBox((35.0, 45.0), (-90.0, -15.0))
    ss.setDepth(args.depth)
    sample_points = M.MOPS_GenerateSeedsPoints(ss)

    # 8. trajectories: a streamline for a single timestep (the reference runs none for a range)
    cfg = M.TrajectorySettings()
    cfg.depth = args.depth
    cfg.deltaT = ONE_HOUR * 1
    cfg.simulationDuration = ONE_DAY * args.day
    cfg.recordT = ONE_HOUR * 6
    cfg.fileName = f"traj_line_{timesteps[0]}"
    if len(timesteps) == 1:
        print("== single timestep [streamline] ==")
        lines = M.MOPS_RunStreamLine(cfg, sample_points)
        if lines:
            stacked = {"points": np.stack([ln["points"] for ln in lines]),
                       "velocity": np.stack([ln["velocity"] for ln in lines])}
            mio.save_trajectory_lines_vtp(cfg.fileName + ".vtp", stacked)
            mio.save_trajectory_lines_txt(cfg.fileName + ".txt", stacked)
            print(f"[✓] Trajectory lines saved to {cfg.fileName}.txt")
        else:
            print(f"[Error] Unable to open file for writing: {cfg.fileName}.txt", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
