"""pyMOPS-compatible Python API (mops_amd/pyMOPS.py), written the way the
reference's Python tutorials use pyMOPS (bindings.cpp:281-455)."""
import numpy as np
import pytest


def test_generate_seeds_points_lattice():
    from mops_amd import pyMOPS, synth
    s = pyMOPS.SeedsSettings()
    s.setSeedsRange((11, 11))
    s.setGeoBox((-40.0, 40.0), (-60.0, 60.0))
    s.setDepth(800.0)
    pts = pyMOPS.MOPS_GenerateSeedsPoints(s)
    assert pts.shape == (100, 3)               # exclusive upper bounds: 11x11 -> 10x10
    assert np.allclose(pts, synth.lattice_seeds(11, 11, (-40.0, 40.0), (-60.0, 60.0)), rtol=0, atol=1e-6)
    with pytest.raises(RuntimeError):
        s.setSeedsRange((1, 2, 3))


def test_shape_error_and_state_errors():
    from mops_amd import pyMOPS
    cfg = pyMOPS.TrajectorySettings()
    assert cfg.methodType == pyMOPS.CalcMethodType.kEuler        # reference default
    with pytest.raises(RuntimeError, match=r"\(N, 3\)"):
        pyMOPS.MOPS_RunStreamLine(cfg, np.zeros((4, 2)))
    pyMOPS._app = pyMOPS._App()
    with pytest.raises(SystemExit):
        pyMOPS.MOPS_End()                                         # not configuring -> exit(1)
    assert pyMOPS.MOPS_RunStreamLine(cfg, np.zeros((4, 3))) == []  # no active field -> Error + []


def _setup(mesh, snaps):
    from mops_amd import pyMOPS as M
    G, A = M.GridAttributeType, M.AttributeType
    M.MOPS_Init("gpu")
    M.MOPS_Begin()
    g = M.MPASOGrid()
    g.setGridAttribute(G.kCellSize, mesh.nCells)
    g.setGridAttribute(G.kVertexSize, mesh.nVertices)
    g.setGridAttribute(G.kMaxEdgesSize, mesh.maxEdges)
    g.setGridAttributesVec3(G.kCellCoord, mesh.cellCoord)
    g.setGridAttributesVec3(G.kVertexCoord, mesh.vertexCoord)
    g.setGridAttributesInt(G.kNumberVertexOnCell, mesh.nEdgesOnCell)
    g.setGridAttributesInt(G.kVerticesOnCell, mesh.verticesOnCell)
    g.setGridAttributesInt(G.kCellsOnCell, mesh.cellsOnCell)
    g.setGridAttributesInt(G.kCellsOnVertex, mesh.cellsOnVertex)
    M.MOPS_AddGridMesh(g)
    for t, s in enumerate(snaps):
        sol = M.MPASOSolution()
        sol.setTimestep(t)
        sol.setAttribute(G.kVertLevels, mesh.nVertLevels)
        sol.setAttribute(G.kVertLevelsP1, mesh.nVertLevels + 1)
        sol.setAttributesDouble(A.kLayerThickness, s.layerThickness)
        sol.setAttributesDouble(A.kBottomDepth, s.bottomDepth)
        sol.setAttributesDouble(A.kZonalVelocity, s.zonalVelocity)
        sol.setAttributesDouble(A.kMeridionalVelocity, s.meridionalVelocity)
        sol.cellVertVelocity_vec = s.vertVelocityTop
        M.MOPS_AddAttribute(t, sol)
    M.MOPS_End()
    return M


@pytest.mark.gpu
def test_pymops_matches_oracle(engine_lib, oracle_lib, gpu, small_case):
    from mops_amd import synth
    mesh, s0, s1 = small_case
    M = _setup(mesh, (s0, s1))
    seeds = synth.uniform_band_seeds(150, seed=33)
    cfg = M.TrajectorySettings()
    cfg.deltaT, cfg.simulationDuration, cfg.recordT, cfg.depth = 600, 86400, 7200, 250.0
    cfg.methodType = M.CalcMethodType.kRK4
    depths = np.linspace(10.0, 900.0, len(seeds)).astype(np.float32)
    cfg.particle_depths = list(depths)
    M.MOPS_ActiveAttribute(0)
    sl = M.MOPS_RunStreamLine(cfg, seeds)
    M.MOPS_ActiveAttribute(0, 1)
    before = seeds.copy()
    pl = M.MOPS_RunPathLine(cfg, seeds)
    assert np.array_equal(seeds, before)            # pybind copies: the numpy input is not modified
    d0, d1 = oracle_lib.preprocess(mesh, s0), oracle_lib.preprocess(mesh, s1)
    rs = oracle_lib.run(mesh, d0, None, seeds, depths=depths, delta_t=600, duration=86400, record_t=7200,
                        euler=False)
    rp = oracle_lib.run(mesh, d0, d1, seeds, depths=depths, delta_t=600, duration=86400, record_t=7200, euler=False)
    assert len(sl) == len(pl) == len(seeds)
    assert set(sl[0]) == {"lineID", "points", "velocity"}
    assert set(pl[0]) == {"lineID", "points", "velocity", "temperature", "salinity", "lastPoint", "depth"}
    for i in range(len(seeds)):
        assert sl[i]["lineID"] == i and pl[i]["lineID"] == i
        assert np.array_equal(sl[i]["points"], rs["points"][i])
        assert np.array_equal(sl[i]["velocity"], rs["velocity"][i])
        assert np.array_equal(pl[i]["points"], rp["points"][i])
        assert np.array_equal(pl[i]["velocity"], rp["velocity"][i])
        assert np.array_equal(pl[i]["temperature"], rp["temperature"][i])
        assert np.array_equal(pl[i]["lastPoint"], rp["lastPoint"][i])
        assert pl[i]["depth"] == float(depths[i])


@pytest.mark.gpu
def test_pymops_normal_velocity_takes_the_rbf_path(engine_lib, oracle_lib, gpu):
    """A solution given AttributeType.kNormalVelocity and no zonal/meridional velocity (plus the grid's
    edges) is reconstructed by the RBF path (MPASOSolution::calcCellCenterVelocity); the streamline
    on it equals the oracle's on the oracle's RBF-derived field."""
    from mops_amd import pyMOPS as M, synth
    mesh = synth.make_mesh(16, n_levels=10, flips=40)
    s = synth.make_snapshot(mesh, normal_velocity=True)
    G, A = M.GridAttributeType, M.AttributeType
    M.MOPS_Init("gpu")
    M.MOPS_Begin()
    g = M.MPASOGrid()
    g.setGridAttribute(G.kCellSize, mesh.nCells)
    g.setGridAttribute(G.kVertexSize, mesh.nVertices)
    g.setGridAttribute(G.kMaxEdgesSize, mesh.maxEdges)
    g.setGridAttribute(G.kEdgeSize, mesh.nEdges)
    g.setGridAttributesVec3(G.kCellCoord, mesh.cellCoord)
    g.setGridAttributesVec3(G.kVertexCoord, mesh.vertexCoord)
    g.setGridAttributesVec3(G.kEdgeCoord, mesh.edgeCoord)
    g.setGridAttributesInt(G.kNumberVertexOnCell, mesh.nEdgesOnCell)
    g.setGridAttributesInt(G.kVerticesOnCell, mesh.verticesOnCell)
    g.setGridAttributesInt(G.kCellsOnCell, mesh.cellsOnCell)
    g.setGridAttributesInt(G.kCellsOnVertex, mesh.cellsOnVertex)
    g.setGridAttributesInt(G.kEdgesOnCell, mesh.edgesOnCell)
    g.setGridAttributesInt(G.kCellsOnEdge, mesh.cellsOnEdge)
    M.MOPS_AddGridMesh(g)
    sol = M.MPASOSolution()
    sol.setTimestep(0)
    sol.setAttribute(G.kVertLevels, mesh.nVertLevels)
    sol.setAttribute(G.kVertLevelsP1, mesh.nVertLevels + 1)
    sol.setAttributesDouble(A.kLayerThickness, s.layerThickness)
    sol.setAttributesDouble(A.kBottomDepth, s.bottomDepth)
    sol.setAttributesDouble(A.kNormalVelocity, s.normalVelocity)
    sol.cellVertVelocity_vec = s.vertVelocityTop
    M.MOPS_AddAttribute(0, sol)
    M.MOPS_End()
    M.MOPS_ActiveAttribute(0)
    seeds = synth.uniform_band_seeds(120, seed=5)
    cfg = M.TrajectorySettings()
    cfg.deltaT, cfg.simulationDuration, cfg.recordT, cfg.depth = 600, 43200, 3600, 300.0
    lines = M.MOPS_RunStreamLine(cfg, seeds)
    ref = oracle_lib.run(mesh, oracle_lib.preprocess(mesh, s, velocity="rbf"), None, seeds, depth=300.0,
                         delta_t=600, duration=43200, record_t=3600, euler=True)
    for i in range(len(seeds)):
        assert np.array_equal(lines[i]["points"], ref["points"][i], equal_nan=True)
        assert np.array_equal(lines[i]["velocity"], ref["velocity"][i], equal_nan=True)
