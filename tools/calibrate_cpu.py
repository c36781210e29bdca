"""Calibrate the CPU port (oracle/) against the reference's own TBB path.

SURVEY.md §6 timed the reference's TBB StreamLine itself (built with stub headers during the survey,
in this container: Intel Xeon, 8 cores) on a 236 000-cell / 60-level synthetic Voronoi mesh, 20 000
particles, dt 120 s, 1 day:
    Euler 0.710 us/particle-step on 1 core (run-to-run 0.71-0.78), 0.101 on 8 threads;
    RK4   1.38  us/particle-step on 1 core,                         0.177 on 8 threads.
The reference cannot be rebuilt here under this round's rules (it needs stand-ins for TBB / netCDF /
ftk headers), so the calibration runs the port on the same shape -- the EC30to60-class mesh
(235 567 cells, 60 levels), 20 000 particles, dt 120 s, 1 day, in this same container -- and divides.
The ratio says how the bench's cpu_baseline (the port on the GPU box's cores) relates to what the
reference's TBB path would do there.

    python tools/calibrate_cpu.py  > profiles/r03/cpu_calibration.json
"""
import json
import os
import platform
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REFERENCE_US = {("euler", 1): 0.710, ("euler", 8): 0.101, ("rk4", 1): 1.38, ("rk4", 8): 0.177}


def main():
    import bench
    from mops_amd import synth
    from oracle import oracle as O
    mesh = synth.make_mesh(158, n_levels=60)
    snap = synth.make_snapshot(mesh)
    d = O.preprocess(mesh, snap)
    seeds = bench.make_seeds(20_000, 0)
    cells = O.knn(mesh, seeds)
    out = {"mesh": {"cells": mesh.nCells, "levels": mesh.nVertLevels}, "particles": len(seeds), "dt": 120,
           "duration": 86400, "cpu": platform.processor() or platform.machine(), "os_cpu_count": os.cpu_count(),
           "runs": []}
    for method in ("euler", "rk4"):
        for threads in (1, 8):
            best = None
            for _ in range(2):
                t = time.perf_counter()
                r = O.run(mesh, d, None, seeds, depth=800.0, delta_t=120, duration=86400, record_t=3600,
                          euler=(method == "euler"), cells=cells, n_threads=threads, finalize=False)
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            death = r["death"].astype(np.int64)
            nominal = len(seeds) * 720
            attempted = int(np.where(death < 0, 720, death + 1).sum())
            us = best / nominal * 1e6  # the survey quotes per nominal particle-step
            ref = REFERENCE_US[(method, threads)]
            out["runs"].append({"method": method, "threads": threads, "seconds": best,
                                "port_us_per_nominal_pstep": us, "attempted_psteps": attempted,
                                "reference_us_per_pstep_survey": ref, "port_speed_over_reference": ref / us})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
