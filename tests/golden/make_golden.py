"""Writes the committed golden fixtures under tests/golden/.

1. remove_nan_cases.json -- the four RemoveNaNTrajectoriesAndReindex cases of
   the reference's own test (test/test_trajector.cpp:26-194): inputs built by
   its make_line() helper (velocity {1,2,3}, temperature 10, salinity 20,
   lineID 42) and the outputs its REQUIREs pin.  `asserted` lists the fields
   the reference test checks; the remaining expected values follow from
   TrajectoryCommon.h:57-129 and are marked "derived".
2. gauss_kat.json -- Interpolator::gauss_elimination_fixed known answer
   (test/test_gaussian.cpp:9-27): x = {4.75, 0.5, 6.0}, tol 1e-6.
3. oracle_small.npz -- outputs of the CPU oracle on a small synthetic case
   (regression vectors for the oracle and the GPU engine; NOT a reference
   pin -- the reference cannot be built here).

Run: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

NAN = float("nan")


def remove_nan_cases():
    def line(pts):
        n = len(pts)
        return dict(points=pts, velocity=[[1.0, 2.0, 3.0]] * n, temperature=[10.0] * n, salinity=[20.0] * n,
                    lineID=42)

    cases = []
    # Case 1: first point NaN -> every point := first point (NaN x), velocity 0
    c1 = line([[NAN, 0.0, 0.0], [5.0, 6.0, 7.0], [8.0, 9.0, 10.0], [11.0, 12.0, 13.0]])
    cases.append(dict(name="case1_first_nan", input=c1,
                      expected=dict(points=[[NAN, 0.0, 0.0]] * 4, velocity=[[0.0, 0.0, 0.0]] * 4,
                                    temperature=[10.0] * 4, salinity=[20.0] * 4, lastPoint=[NAN, 0.0, 0.0],
                                    lineID=0),
                      asserted=["len", "points.x_is_nan", "velocity"]))
    # Case 2: NaN at index 1 -> pad with point 0, velocity[0] := 0
    c2 = line([[1.0, 2.0, 3.0], [NAN, 0.0, 0.0], [7.0, 8.0, 9.0], [10.0, 11.0, 12.0]])
    cases.append(dict(name="case2_second_nan", input=c2,
                      expected=dict(points=[[1.0, 2.0, 3.0]] * 4, velocity=[[0.0, 0.0, 0.0]] * 4,
                                    temperature=[10.0] * 4, salinity=[20.0] * 4, lastPoint=[1.0, 2.0, 3.0],
                                    lineID=0),
                      asserted=["len", "lineID", "points", "velocity", "lastPoint"]))
    # Case 3: NaN at index 2 of 5
    c3 = line([[10.0, 1.0, 1.0], [11.0, 2.0, 2.0], [NAN, 0.0, 0.0], [13.0, 4.0, 4.0], [14.0, 5.0, 5.0]])
    cases.append(dict(name="case3_middle_nan", input=c3,
                      expected=dict(points=[[10.0, 1.0, 1.0], [11.0, 2.0, 2.0], [11.0, 2.0, 2.0], [11.0, 2.0, 2.0],
                                            [11.0, 2.0, 2.0]],
                                    velocity=[[1.0, 2.0, 3.0]] + [[0.0, 0.0, 0.0]] * 4,
                                    temperature=[10.0] * 5, salinity=[20.0] * 5, lastPoint=[11.0, 2.0, 2.0],
                                    lineID=0),
                      asserted=["len", "points[0:2]", "points[2:]", "velocity[1:]", "lastPoint.xy"]))
    # Case 4: all valid -> unchanged
    c4 = line([[1.0, 1.0, 1.0], [2.0, 2.0, 2.0], [3.0, 3.0, 3.0], [4.0, 4.0, 4.0]])
    cases.append(dict(name="case4_all_valid", input=c4,
                      expected=dict(points=c4["points"], velocity=[[1.0, 2.0, 3.0]] * 4, temperature=[10.0] * 4,
                                    salinity=[20.0] * 4, lastPoint=[4.0, 4.0, 4.0], lineID=0),
                      asserted=["len", "points.x", "velocity", "lastPoint"]))
    return dict(source="reference test/test_trajector.cpp:26-194 (RemoveNaNTrajectoriesAndReindex)",
                cases=cases)


def gauss_kat():
    return dict(source="reference test/test_gaussian.cpp:9-27 (Interpolator::gauss_elimination_fixed)",
                A=[[2.0, 3.0, -1.0], [4.0, 4.0, -3.0], [-2.0, 3.0, 2.0]], b=[5.0, 3.0, 4.0],
                expected=[4.75, 0.5, 6.0], tol=1e-6)


def oracle_small():
    from mops_amd import synth
    from oracle import oracle as O
    mesh = synth.make_mesh(8, n_levels=10)
    s0 = synth.make_snapshot(mesh, timestep=0)
    s1 = synth.make_snapshot(mesh, timestep=1, phase=0.35)
    d0, d1 = O.preprocess(mesh, s0), O.preprocess(mesh, s1)
    seeds = synth.lattice_seeds(9, 9, (-40.0, 40.0), (-60.0, 60.0))
    out = dict(seeds=seeds, freq=np.array(8), levels=np.array(10))
    for name, back, euler in (("stream_euler", None, True), ("stream_rk4", None, False),
                              ("path_euler", d1, True), ("path_rk4", d1, False)):
        r = O.run(mesh, d0, back, seeds, depth=500.0, delta_t=300, duration=21600, record_t=3600, euler=euler)
        out[f"{name}_points"] = r["points"]
        out[f"{name}_velocity"] = r["velocity"]
        out[f"{name}_death"] = r["death"]
        out[f"{name}_depth"] = r["final_depth"]
        out[f"{name}_cells"] = r["cells"]
    return out


def main():
    with open(os.path.join(HERE, "remove_nan_cases.json"), "w") as f:
        json.dump(remove_nan_cases(), f, indent=1)
    with open(os.path.join(HERE, "gauss_kat.json"), "w") as f:
        json.dump(gauss_kat(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "oracle_small.npz"), **oracle_small())
    print("golden fixtures written")


if __name__ == "__main__":
    main()
