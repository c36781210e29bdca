// mops_api_demo.cpp -- the reference tutorial's call sequence on the MI355X
// engine (reference: tutorials/ streamline/pathline examples driving
// include/api/MOPS.h).  Reads a case written by tests/test_cpp_api.py as raw
// little-endian arrays, runs StreamLine then PathLine through the MOPS::
// API, and writes the lines back as raw arrays.
//
//   mops_api_demo <case_dir>
//
// case_dir/dims.txt : C V maxE L N deltaT duration recordT depth method
// inputs            : nEdgesOnCell verticesOnCell cellsOnCell cellsOnVertex
//                     (u64), cellCoord vertexCoord seeds (f64 xyz),
//                     {layerThickness,bottomDepth,zonal,meridional,vvel}_{0,1} (f64)
// outputs           : stream_{points,velocity}.f64, path_{points,velocity,
//                     temperature,salinity,last}.f64, path_seeds_after.f64
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "mops/MOPS.h"

template <class T>
static std::vector<T> load(const std::string& path, size_t n) {
    std::vector<T> v(n);
    std::ifstream f(path, std::ios::binary);
    if (!f || !f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(n * sizeof(T)))) {
        std::cerr << "cannot read " << path << "\n";
        std::exit(2);
    }
    return v;
}

template <class T>
static void save(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

static void save_lines(const std::string& dir, const std::string& tag, const std::vector<MOPS::TrajectoryLine>& lines,
                       bool attrs) {
    std::vector<double> pts, vel, tmp, sal, last;
    for (const auto& l : lines) {
        for (const auto& p : l.points) pts.insert(pts.end(), {p.x, p.y, p.z});
        for (const auto& v : l.velocity) vel.insert(vel.end(), {v.x, v.y, v.z});
        tmp.insert(tmp.end(), l.temperature.begin(), l.temperature.end());
        sal.insert(sal.end(), l.salinity.begin(), l.salinity.end());
        last.insert(last.end(), {l.lastPoint.x, l.lastPoint.y, l.lastPoint.z});
    }
    save(dir + "/" + tag + "_points.f64", pts.data(), pts.size());
    save(dir + "/" + tag + "_velocity.f64", vel.data(), vel.size());
    save(dir + "/" + tag + "_last.f64", last.data(), last.size());
    if (attrs) {
        save(dir + "/" + tag + "_temperature.f64", tmp.data(), tmp.size());
        save(dir + "/" + tag + "_salinity.f64", sal.data(), sal.size());
    }
}

int main(int argc, char** argv) {
    using namespace MOPS;
    if (argc < 2) {
        std::cerr << "usage: mops_api_demo <case_dir>\n";
        return 2;
    }
    const std::string dir = argv[1];
    size_t C, V, maxE, L, N, dt, dur, rT;
    double depth;
    int method;
    {
        std::ifstream f(dir + "/dims.txt");
        if (!(f >> C >> V >> maxE >> L >> N >> dt >> dur >> rT >> depth >> method)) {
            std::cerr << "bad dims.txt\n";
            return 2;
        }
    }
    auto as_vec3 = [](const std::vector<double>& a) {
        std::vector<vec3> v(a.size() / 3);
        for (size_t i = 0; i < v.size(); ++i) v[i] = {a[3 * i], a[3 * i + 1], a[3 * i + 2]};
        return v;
    };

    MOPS_Init("gpu");
    MOPS_Begin();
    auto grid = std::make_shared<MPASOGrid>();
    grid->setGridAttribute(GridAttributeType::kCellSize, (int)C);
    grid->setGridAttribute(GridAttributeType::kVertexSize, (int)V);
    grid->setGridAttribute(GridAttributeType::kMaxEdgesSize, (int)maxE);
    grid->setGridAttributesVec3(GridAttributeType::kCellCoord, as_vec3(load<double>(dir + "/cellCoord", C * 3)));
    grid->setGridAttributesVec3(GridAttributeType::kVertexCoord, as_vec3(load<double>(dir + "/vertexCoord", V * 3)));
    grid->setGridAttributesInt(GridAttributeType::kNumberVertexOnCell, load<size_t>(dir + "/nEdgesOnCell", C));
    grid->setGridAttributesInt(GridAttributeType::kVerticesOnCell, load<size_t>(dir + "/verticesOnCell", C * maxE));
    grid->setGridAttributesInt(GridAttributeType::kCellsOnCell, load<size_t>(dir + "/cellsOnCell", C * maxE));
    grid->setGridAttributesInt(GridAttributeType::kCellsOnVertex, load<size_t>(dir + "/cellsOnVertex", V * 3));
    MOPS_AddGridMesh(grid);
    for (int t = 0; t < 2; ++t) {
        auto sol = std::make_shared<MPASOSolution>();
        const std::string s = "_" + std::to_string(t);
        sol->setTimestep(t);
        sol->setAttribute(GridAttributeType::kVertLevels, (int)L);
        sol->setAttribute(GridAttributeType::kVertLevelsP1, (int)L + 1);
        sol->setAttributesDouble(AttributeType::kLayerThickness, load<double>(dir + "/layerThickness" + s, C * L));
        sol->setAttributesDouble(AttributeType::kBottomDepth, load<double>(dir + "/bottomDepth" + s, C));
        sol->setAttributesDouble(AttributeType::kZonalVelocity, load<double>(dir + "/zonal" + s, C * L));
        sol->setAttributesDouble(AttributeType::kMeridionalVelocity, load<double>(dir + "/meridional" + s, C * L));
        sol->cellVertVelocity_vec = load<double>(dir + "/vvel" + s, C * (L + 1));
        MOPS_AddAttribute(t, sol);
    }
    MOPS_End();

    std::vector<CartesianCoord> seeds = as_vec3(load<double>(dir + "/seeds", N * 3));
    TrajectorySettings cfg;
    cfg.deltaT = dt;
    cfg.simulationDuration = dur;
    cfg.recordT = rT;
    cfg.depth = (float)depth;
    cfg.directionType = CalcDirection::kForward;
    cfg.methodType = method == 1 ? CalcMethodType::kEuler : CalcMethodType::kRK4;

    MOPS_ActiveAttribute(0);
    auto stream = MOPS_RunStreamLine(&cfg, seeds);
    save_lines(dir, "stream", stream, false);

    MOPS_ActiveAttribute(0, 1);
    auto path = MOPS_RunPathLine(&cfg, seeds);
    save_lines(dir, "path", path, true);
    std::vector<double> after;
    for (const auto& p : seeds) after.insert(after.end(), {p.x, p.y, p.z});
    save(dir + "/path_seeds_after.f64", after.data(), after.size());

    SamplingSettings sampling;
    sampling.setSamplingRegion({11, 11}, {-40.0, 40.0}, {-60.0, 60.0}, 800.0);
    std::vector<CartesianCoord> lattice;
    MOPS_GenerateSamplePoints(&sampling, lattice);
    save(dir + "/lattice.f64", reinterpret_cast<const double*>(lattice.data()), lattice.size() * 3);

    std::printf("lines %zu %zu points %zu lattice %zu\n", stream.size(), path.size(),
                stream.empty() ? (size_t)0 : stream[0].points.size(), lattice.size());
    MOPS_PrintTimingSummary();
    MOPS_Finalize();
    return 0;
}
