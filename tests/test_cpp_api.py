"""The MOPS:: C++ API (include/mops/MOPS.h) driven the way the reference's
tutorials drive include/api/MOPS.h: Init -> Begin -> AddGridMesh ->
AddAttribute x2 -> End -> ActiveAttribute -> RunStreamLine / RunPathLine ->
GenerateSamplePoints.  The demo program is compiled with g++ against the
engine library; its output lines are checked against the CPU oracle."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO_SRC = os.path.join(ROOT, "examples", "mops_api_demo.cpp")


def _compile(engine_lib, out_dir):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = os.path.join(str(out_dir), "mops_api_demo")
    libdir = os.path.join(ROOT, "mops_amd", "lib")
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), DEMO_SRC,
           "-L" + libdir, "-lmops_traj", "-Wl,-rpath," + libdir, "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_cpp_api_compiles_and_links(engine_lib, tmp_path):
    """The header is self-contained C++17 and every MOPS:: symbol resolves
    in libmops_traj.so (no GPU needed to link)."""
    exe = _compile(engine_lib, tmp_path)
    assert os.path.exists(exe)


def _write_case(d, mesh, snaps, seeds, dt, dur, rT, depth, method):
    L = mesh.nVertLevels
    with open(os.path.join(d, "dims.txt"), "w") as f:
        f.write(f"{mesh.nCells} {mesh.nVertices} {mesh.maxEdges} {L} {len(seeds)} {dt} {dur} {rT} {depth} {method}\n")
    arrays = dict(nEdgesOnCell=mesh.nEdgesOnCell, verticesOnCell=mesh.verticesOnCell, cellsOnCell=mesh.cellsOnCell,
                  cellsOnVertex=mesh.cellsOnVertex, cellCoord=mesh.cellCoord, vertexCoord=mesh.vertexCoord,
                  seeds=seeds)
    for t, s in enumerate(snaps):
        arrays.update({f"layerThickness_{t}": s.layerThickness, f"bottomDepth_{t}": s.bottomDepth,
                       f"zonal_{t}": s.zonalVelocity, f"meridional_{t}": s.meridionalVelocity,
                       f"vvel_{t}": s.vertVelocityTop})
    for k, a in arrays.items():
        a = np.ascontiguousarray(a)
        a = a.astype(np.uint64) if a.dtype.kind in "iu" else a.astype(np.float64)
        a.tofile(os.path.join(d, k))


def _read(d, name, shape):
    return np.fromfile(os.path.join(d, name), dtype=np.float64).reshape(shape)


@pytest.mark.gpu
@pytest.mark.parametrize("method", [1, 0], ids=["euler", "rk4"])
def test_cpp_api_matches_oracle(engine_lib, oracle_lib, gpu, small_case, tmp_path, method):
    from mops_amd import synth
    mesh, s0, s1 = small_case
    seeds = synth.uniform_band_seeds(200, seed=21)
    dt, dur, rT, depth = 300, 43200, 3600, 400.0
    exe = _compile(engine_lib, tmp_path)
    d = str(tmp_path)
    _write_case(d, mesh, (s0, s1), seeds, dt, dur, rT, depth, method)
    r = subprocess.run([exe, d], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    N, P = len(seeds), dur // rT + 1
    d0, d1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    euler = method == 1
    ref_s = oracle_lib.run(mesh, d0, None, seeds, depth=depth, delta_t=dt, duration=dur, record_t=rT, euler=euler)
    ref_p = oracle_lib.run(mesh, d0, d1, seeds, depth=depth, delta_t=dt, duration=dur, record_t=rT, euler=euler)
    # bit-exact: same FP64 operation order, no contraction
    assert np.array_equal(_read(d, "stream_points.f64", (N, P, 3)), ref_s["points"])
    assert np.array_equal(_read(d, "stream_velocity.f64", (N, P, 3)), ref_s["velocity"])
    assert np.array_equal(_read(d, "stream_last.f64", (N, 3)), ref_s["lastPoint"])
    assert np.array_equal(_read(d, "path_points.f64", (N, P, 3)), ref_p["points"])
    assert np.array_equal(_read(d, "path_velocity.f64", (N, P, 3)), ref_p["velocity"])
    assert np.array_equal(_read(d, "path_temperature.f64", (N, P)), ref_p["temperature"])
    assert np.array_equal(_read(d, "path_salinity.f64", (N, P)), ref_p["salinity"])
    # MOPSApp::runPathLine overwrites sample_points with lastPoint (MOPSApp.cpp:287-290)
    assert np.array_equal(_read(d, "path_seeds_after.f64", (N, 3)), ref_p["lastPoint"])
    lat = _read(d, "lattice.f64", (-1, 3))
    # host libm vs numpy sin/cos may differ in the last ulp
    assert np.allclose(lat, synth.lattice_seeds(11, 11, (-40.0, 40.0), (-60.0, 60.0)), rtol=0, atol=1e-6)
