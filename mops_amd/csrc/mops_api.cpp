// mops_api.cpp -- the MOPS:: C++ operator API (include/mops/MOPS.h) on top
// of the C ABI.  Mirrors the reference's MOPS.cpp / MOPSApp.cpp state machine
// (src/Core/MOPS.cpp:10-71, src/Core/MOPSApp.cpp:34-337): one global app,
// Init -> Begin -> AddGridMesh -> AddAttribute* -> End -> ActiveAttribute ->
// RunStreamLine / RunPathLine.  Every trajectory computation goes to the HIP
// engine; this file only marshals host containers.
#include "mops/MOPS.h"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <stdexcept>

namespace MOPS {
static_assert(sizeof(CartesianCoord) == 3 * sizeof(double), "CartesianCoord is packed xyz (host <-> device copies)");
namespace {

void Error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::fprintf(stderr, "[Error]: ");
    std::vfprintf(stderr, fmt, ap);
    std::fprintf(stderr, "\n");
    va_end(ap);
}

// ---- TimerManager (src/Utils/Timer.hpp:17-216, categories only) ----------
struct Timing {
    std::map<std::string, double> by_category;
    std::vector<std::pair<std::string, double>> records;
    void add(const std::string& name, const std::string& cat, double ms) {
        by_category[cat] += ms;
        records.emplace_back(name, ms);
    }
};
Timing g_timing;

struct ScopedTimer {
    std::string name, cat;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ScopedTimer(std::string n, std::string c) : name(std::move(n)), cat(std::move(c)) {}
    ~ScopedTimer() {
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        g_timing.add(name, cat, ms);
    }
};

enum class State { Idle, Configuring, Ready };

struct App {
    State state = State::Idle;
    std::shared_ptr<MPASOGrid> grid;
    std::map<int, std::shared_ptr<MPASOSolution>> sols;
    mops_mesh* mesh = nullptr;
    std::map<int, mops_field*> fields;
    mops_field* front = nullptr;
    mops_field* back = nullptr;

    void release() {
        for (auto& kv : fields) mops_field_destroy(kv.second);
        fields.clear();
        if (mesh) mops_mesh_destroy(mesh);
        mesh = nullptr;
        front = back = nullptr;
    }
    // No device frees here: g_app is destroyed during static destruction, when the
    // HIP runtime may already be torn down.  Device state is released by MOPS_Init
    // (re-initialisation) and MOPS_Finalize; whatever is left at exit is reclaimed
    // with the process.
    ~App() = default;
};
App g_app;

void check(mops_status st, const char* what) {
    if (st != MOPS_OK) throw std::runtime_error(std::string(what) + ": " + mops_last_error());
}

mops_field* make_field(const MPASOSolution& s) {
    mops_snapshot_desc d{};
    d.timestep = s.mTimesteps;
    d.h_layer_thickness = s.cellLayerThickness_vec.empty() ? nullptr : s.cellLayerThickness_vec.data();
    d.h_bottom_depth = s.cellBottomDepth_vec.empty() ? nullptr : s.cellBottomDepth_vec.data();
    d.h_surface_height = s.cellSurfaceHeight_vec.empty() ? nullptr : s.cellSurfaceHeight_vec.data();
    d.h_zonal_velocity = s.cellZonalVelocity_vec.empty() ? nullptr : s.cellZonalVelocity_vec.data();
    d.h_meridional_velocity = s.cellMeridionalVelocity_vec.empty() ? nullptr : s.cellMeridionalVelocity_vec.data();
    d.h_vert_velocity_top = s.cellVertVelocity_vec.empty() ? nullptr : s.cellVertVelocity_vec.data();
    d.h_normal_velocity = s.cellNormalVelocity_vec.empty() ? nullptr : s.cellNormalVelocity_vec.data();
    mops_field* f = nullptr;
    check(mops_field_create(g_app.mesh, &d, nullptr, &f), "mops_field_create");
    return f;
}

std::vector<TrajectoryLine> run(TrajectorySettings* config, std::vector<CartesianCoord>& pts, bool pathline,
                                const char* stage) {
    if (config == nullptr || g_app.front == nullptr || (pathline && g_app.back == nullptr)) {
        Error("[%s] invalid inputs", stage);  // MPASOVisualizerKernels.cpp:659-662
        return {};
    }
    if (pts.empty()) return {};
    if (config->deltaT == 0 || config->recordT == 0 || config->simulationDuration == 0) {
        Error("[%s] invalid trajectory settings", stage);  // :666-669
        return {};
    }
    const int64_t n = (int64_t)pts.size();
    const bool per_particle = config->hasPerParticleDepths() && config->particle_depths.size() == pts.size();
    std::vector<float> depths(pts.size(), config->depth);  // BuildEffectiveDepths (TrajectoryCommon.h:29-41)
    if (per_particle) depths = config->particle_depths;
    mops_traj_cfg cfg{(int64_t)config->deltaT, (int64_t)config->simulationDuration, (int64_t)config->recordT,
                      config->directionType == CalcDirection::kForward ? MOPS_FORWARD : MOPS_BACKWARD,
                      config->methodType == CalcMethodType::kEuler ? MOPS_EULER : MOPS_RK4};
    const int64_t K = mops_traj_num_records(&cfg), steps = mops_traj_num_steps(&cfg);
    std::vector<TrajectoryLine> lines((size_t)n);
    for (int64_t i = 0; i < n; ++i) {  // InitTrajectoryLines (:43-55)
        auto& l = lines[(size_t)i];
        l.lineID = (int)i;
        l.points = {pts[(size_t)i]};
        l.lastPoint = pts[(size_t)i];
        l.duration = (double)config->simulationDuration;
        l.timestamp = (double)config->deltaT;
        l.depth = depths[(size_t)i];
    }
    if (K <= 0 || steps <= 0) {
        Error("[%s] invalid integration steps", stage);  // :709-712 returns the seed-only lines
        return lines;
    }
    const int64_t P = K + 1;
    std::vector<double> hp((size_t)(n * P * 3)), hv((size_t)(n * P * 3)), ht((size_t)(n * P)), hs((size_t)(n * P)),
        hl((size_t)(n * 3));
    check(mops_run_trajectories(g_app.mesh, g_app.front, pathline ? g_app.back : nullptr, &cfg, n,
                                reinterpret_cast<const double*>(pts.data()), depths.data(), config->depth, nullptr,
                                hp.data(), hv.data(), ht.data(), hs.data(), hl.data(), nullptr, nullptr, nullptr,
                                nullptr),
          "mops_run_trajectories");
    for (int64_t i = 0; i < n; ++i) {  // FinalizeTrajectoryLines[WithAttrs] + RemoveNaN (device-side)
        auto& l = lines[(size_t)i];
        l.points.resize((size_t)P);
        l.velocity.resize((size_t)P);
        l.temperature.resize((size_t)P);
        l.salinity.resize((size_t)P);
        for (int64_t j = 0; j < P; ++j) {
            const size_t q = (size_t)((i * P + j) * 3);
            l.points[(size_t)j] = {hp[q], hp[q + 1], hp[q + 2]};
            l.velocity[(size_t)j] = {hv[q], hv[q + 1], hv[q + 2]};
            l.temperature[(size_t)j] = ht[(size_t)(i * P + j)];
            l.salinity[(size_t)j] = hs[(size_t)(i * P + j)];
        }
        l.lastPoint = {hl[(size_t)(3 * i)], hl[(size_t)(3 * i + 1)], hl[(size_t)(3 * i + 2)]};
    }
    return lines;
}

}  // namespace

// ---- data model setters (MPASOGrid.cpp:82-188, MPASOSolution.cpp:1145-1210) ----
void MPASOGrid::setGridAttribute(GridAttributeType type, int val) {
    switch (type) {
        case GridAttributeType::kCellSize: mCellsSize = val; break;
        case GridAttributeType::kEdgeSize: mEdgesSize = val; break;
        case GridAttributeType::kVertexSize: mVertexSize = val; break;
        case GridAttributeType::kMaxEdgesSize: mMaxEdgesSize = val; break;
        case GridAttributeType::kVertLevels: mVertLevels = val; break;
        case GridAttributeType::kVertLevelsP1: mVertLevelsP1 = val; break;
        default: Error("[MPASOGrid]::Invalid GridAttributeType"); break;
    }
}
void MPASOGrid::setGridAttributesVec3(GridAttributeType type, const std::vector<vec3>& vec) {
    switch (type) {
        case GridAttributeType::kVertexCoord: vertexCoord_vec = vec; break;
        case GridAttributeType::kCellCoord: cellCoord_vec = vec; break;
        case GridAttributeType::kEdgeCoord: edgeCoord_vec = vec; break;
        default: std::cout << "Error: Invalid GridAttributeType" << std::endl;
    }
}
void MPASOGrid::setGridAttributesVec2(GridAttributeType type, const std::vector<vec2>& vec) {
    if (type == GridAttributeType::kVertexLatLon) vertexLatLon_vec = vec;
    else std::cout << "Error: Invalid GridAttributeType" << std::endl;
}
void MPASOGrid::setGridAttributesInt(GridAttributeType type, const std::vector<size_t>& vec) {
    switch (type) {
        case GridAttributeType::kVerticesOnCell: verticesOnCell_vec = vec; break;
        case GridAttributeType::kVerticesOnEdge: verticesOnEdge_vec = vec; break;
        case GridAttributeType::kCellsOnVertex: cellsOnVertex_vec = vec; break;
        case GridAttributeType::kCellsOnCell: cellsOnCell_vec = vec; break;
        case GridAttributeType::kNumberVertexOnCell: numberVertexOnCell_vec = vec; break;
        case GridAttributeType::kCellsOnEdge: cellsOnEdge_vec = vec; break;
        case GridAttributeType::kEdgesOnCell: edgesOnCell_vec = vec; break;
        default: std::cout << "Error: Invalid GridAttributeType" << std::endl;
    }
}
void MPASOGrid::setGridAttributesFloat(GridAttributeType type, const std::vector<float>& vec) {
    if (type == GridAttributeType::kCellWeight) cellWeight_vec = vec;
    else std::cout << "Error: Invalid GridAttributeType" << std::endl;
}
bool MPASOGrid::checkAttribute() const {  // MPASOGrid.cpp:516-598
    return mCellsSize != 0 && mVertexSize != 0 && mMaxEdgesSize != 0 && mVertLevels != 0 && mVertLevelsP1 != 0 &&
           !cellCoord_vec.empty() && !vertexCoord_vec.empty() && !verticesOnCell_vec.empty() &&
           !cellsOnVertex_vec.empty() && !cellsOnCell_vec.empty() && !numberVertexOnCell_vec.empty();
}

void MPASOSolution::setAttribute(GridAttributeType type, int val) {
    switch (type) {
        case GridAttributeType::kCellSize: mCellsSize = val; break;
        case GridAttributeType::kEdgeSize: mEdgesSize = val; break;
        case GridAttributeType::kVertexSize: mVertexSize = val; break;
        case GridAttributeType::kMaxEdgesSize: mMaxEdgesSize = val; break;
        case GridAttributeType::kVertLevels: mVertLevels = val; break;
        case GridAttributeType::kVertLevelsP1: mVertLevelsP1 = val; break;
        default: std::cerr << "[Error]: Invalid GridAttributeType" << std::endl; break;
    }
}
void MPASOSolution::setAttributesDouble(AttributeType type, const std::vector<double>& vec) {
    switch (type) {
        case AttributeType::kZTop: cellZTop_vec = vec; break;
        case AttributeType::kLayerThickness: cellLayerThickness_vec = vec; break;
        case AttributeType::kBottomDepth: cellBottomDepth_vec = vec; break;
        case AttributeType::kZonalVelocity: cellZonalVelocity_vec = vec; break;
        case AttributeType::kMeridionalVelocity: cellMeridionalVelocity_vec = vec; break;
        case AttributeType::kNormalVelocity: cellNormalVelocity_vec = vec; break;
        default: std::cerr << "[Error]: Invalid AttributeType" << std::endl; break;
    }
}
void MPASOSolution::setAttributesVec3(AttributeType type, const std::vector<vec3>& vec) {
    if (type == AttributeType::kVelocity) cellCenterVelocity_vec = vec;
    else std::cerr << "[Error]: Invalid AttributeType" << std::endl;
}
bool MPASOSolution::checkAttribute() const {  // MPASOSolution.cpp:1212-1232
    if (cellZTop_vec.empty() && cellLayerThickness_vec.empty()) {
        std::cerr << "[MPASOSolution]::Error: Invalid ZTop Attribute" << std::endl;
        return false;
    }
    return true;
}

// ---- public API (MOPS.cpp) -------------------------------------------------
void MOPS_Init(const char* device) {
    (void)device;
    g_app.release();
    g_app = App();
    hipDeviceProp_t prop{};
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        std::cout << " [ system information ]\nDevice selected : " << prop.name << " (" << prop.gcnArchName
                  << ", HIP engine)\n";
    g_app.grid = std::make_shared<MPASOGrid>();
}

void MOPS_Finalize() {
    g_app.release();
    g_app.sols.clear();
    g_app.state = State::Idle;
}

void MOPS_Begin() { g_app.state = State::Configuring; }

void MOPS_AddGridMesh(std::shared_ptr<MPASOGrid> grid) {
    ScopedTimer t("Preprocessing::addGrid", "Preprocessing");
    g_app.grid = std::move(grid);
}

void MOPS_AddAttribute(int solID, std::shared_ptr<MPASOSolution> sol) {
    ScopedTimer t("Preprocessing::addSol", "Preprocessing");
    if (g_app.sols.count(solID)) return;  // MOPSApp.cpp:82-87
    auto& g = *g_app.grid;
    sol->mCellsSize = g.mCellsSize;       // :92-98
    sol->mEdgesSize = g.mEdgesSize;
    sol->mMaxEdgesSize = g.mMaxEdgesSize;
    sol->mVertexSize = g.mVertexSize;
    g.mVertLevels = sol->mVertLevels;
    g.mVertLevelsP1 = sol->mVertLevelsP1;
    g_app.sols[solID] = std::move(sol);
}

void MOPS_End() {
    if (g_app.state != State::Configuring) {  // MOPS.cpp:31-46
        std::cerr << " [ MOPS is not configuring ]\n";
        std::exit(1);
    }
    bool ok = g_app.grid && g_app.grid->checkAttribute();
    for (auto& kv : g_app.sols) ok = ok && kv.second && kv.second->checkAttribute();
    if (!ok) {
        std::cerr << " [ MOPS is not configured ]\n";
        std::exit(1);
    }
    g_app.state = State::Ready;
    ScopedTimer t("Preprocessing::upload", "Preprocessing");
    const auto& g = *g_app.grid;
    mops_mesh_desc d{};
    d.n_cells = g.mCellsSize;
    d.n_vertices = g.mVertexSize;
    d.max_edges = g.mMaxEdgesSize;
    d.n_vert_levels = g.mVertLevels;
    d.h_n_edges_on_cell = reinterpret_cast<const uint64_t*>(g.numberVertexOnCell_vec.data());
    d.h_vertices_on_cell = reinterpret_cast<const uint64_t*>(g.verticesOnCell_vec.data());
    d.h_cells_on_cell = reinterpret_cast<const uint64_t*>(g.cellsOnCell_vec.data());
    d.h_cells_on_vertex = reinterpret_cast<const uint64_t*>(g.cellsOnVertex_vec.data());
    d.h_cell_coord = reinterpret_cast<const double*>(g.cellCoord_vec.data());
    d.h_vertex_coord = reinterpret_cast<const double*>(g.vertexCoord_vec.data());
    g_app.release();
    check(mops_mesh_create(&d, nullptr, &g_app.mesh), "mops_mesh_create");
    // a solution with edge-normal velocity only (AttributeType::kNormalVelocity) is reconstructed by
    // the RBF path (MPASOSolution::calcCellCenterVelocity), which needs the mesh's edges
    bool rbf = false;
    for (auto& kv : g_app.sols)
        rbf = rbf || ((kv.second->cellZonalVelocity_vec.empty() || kv.second->cellMeridionalVelocity_vec.empty()) &&
                      !kv.second->cellNormalVelocity_vec.empty());
    if (rbf)
        check(mops_mesh_set_edges(g_app.mesh, (int64_t)g.edgeCoord_vec.size(),
                                  reinterpret_cast<const uint64_t*>(g.edgesOnCell_vec.data()),
                                  reinterpret_cast<const uint64_t*>(g.cellsOnEdge_vec.data()),
                                  reinterpret_cast<const double*>(g.edgeCoord_vec.data()), nullptr),
              "mops_mesh_set_edges");
    for (auto& kv : g_app.sols) g_app.fields[kv.first] = make_field(*kv.second);
    if (!g_app.fields.empty()) g_app.front = g_app.fields.begin()->second;  // addField: first map entry
}

void MOPS_ActiveAttribute(int t1, std::optional<int> t2) {  // MOPSApp.cpp:145-169
    g_app.front = g_app.back = nullptr;
    auto it = g_app.fields.find(t1);
    if (it == g_app.fields.end()) {
        Error("[MOPSApp]::activeAttribute: solID %d not found", t1);
        return;
    }
    if (t2.has_value()) {
        auto it2 = g_app.fields.find(t2.value());
        if (it2 == g_app.fields.end()) {
            Error("[MOPSApp]::activeAttribute: solID %d not found", t2.value());
            return;
        }
        g_app.back = it2->second;
    }
    g_app.front = it->second;
}

std::vector<TrajectoryLine> MOPS_RunStreamLine(TrajectorySettings* config, std::vector<CartesianCoord>& sample_points) {
    ScopedTimer t("GPUKernel::StreamLine", "GPUKernel");
    return run(config, sample_points, false, "MI355X::StreamLine");
}

std::vector<TrajectoryLine> MOPS_RunPathLine(TrajectorySettings* config, std::vector<CartesianCoord>& sample_points) {
    ScopedTimer t("GPUKernel::PathLine", "GPUKernel");
    if (g_app.front == nullptr || g_app.back == nullptr) {  // MOPSApp.cpp:259-271
        Error("[MOPSApp]::Sol_Front or Sol_Back is nullptr, please activeAttribute first");
        std::exit(-1);
    }
    auto lines = run(config, sample_points, true, "MI355X::PathLine");
    for (size_t i = 0; i < sample_points.size() && i < lines.size(); ++i)  // :287-290
        sample_points[i] = lines[i].lastPoint;
    return lines;
}

void MOPS_GenerateSamplePoints(SamplingSettings* config, std::vector<CartesianCoord>& points) {
    if (config->isAtCellCenter()) {  // MOPSApp::generateSamplePointsAtCenter
        for (const auto& p : g_app.grid->cellCoord_vec) points.push_back(p);
        return;
    }
    // MPASOVisualizer::GenerateSamplePoint (MPASOVisualizer.cpp:120-149):
    // exclusive upper bounds, accumulated steps, r = 6371010.0f.  Like the
    // reference, the conversion pass runs over the WHOLE vector, so points the
    // caller passed in are re-converted too.
    const double minLat = config->getLatitudeRange().x, maxLat = config->getLatitudeRange().y;
    const double minLon = config->getLongitudeRange().x, maxLon = config->getLongitudeRange().y;
    const double i_step = (maxLat - minLat) / static_cast<double>(config->getSampleRange().x - 1);
    const double j_step = (maxLon - minLon) / static_cast<double>(config->getSampleRange().y - 1);
    for (double i = minLat; i < maxLat; i += i_step)
        for (double j = minLon; j < maxLon; j += j_step) points.push_back({j, i, config->getDepth()});
    const double r = 6371010.0f;
    for (size_t k = 0; k < points.size(); ++k) {
        const double lat = points[k].y * (M_PI / 180.0), lon = points[k].x * (M_PI / 180.0);
        const double ct = std::cos(lat), cp = std::cos(lon), st = std::sin(lat), sp = std::sin(lon);
        points[k] = {r * ct * cp, r * ct * sp, r * st};
    }
}

void MOPS_ResetTiming() { g_timing = Timing(); }
void MOPS_PrintTimingSummary() {
    std::cout << "==== MOPS timing summary (ms) ====\n";
    for (auto& kv : g_timing.by_category) std::cout << "  " << kv.first << ": " << kv.second << "\n";
}
void MOPS_PrintTimingDetailed() {
    std::cout << "==== MOPS timing detailed (ms) ====\n";
    for (auto& r : g_timing.records) std::cout << "  " << r.first << ": " << r.second << "\n";
}
double MOPS_GetCategoryTime(const char* category) {
    auto it = g_timing.by_category.find(category ? category : "Other");
    return it == g_timing.by_category.end() ? 0.0 : it->second;
}
double MOPS_GetTotalTime() {
    double s = 0.0;
    for (auto& kv : g_timing.by_category) s += kv.second;
    return s;
}

// RemoveNaNTrajectoriesAndReindex (src/Common/TrajectoryCommon.h:57-129): every non-empty line
// packed into one device allocation, cleaned by ONE mops_remove_nan_ragged launch, copied back.
std::vector<TrajectoryLine> RemoveNaNTrajectoriesAndReindex(std::vector<TrajectoryLine>& lines) {
    std::vector<TrajectoryLine*> keep;  // empty lines are dropped (:84-86)
    keep.reserve(lines.size());
    std::vector<int64_t> off(1, 0);
    for (auto& l : lines) {
        const size_t P = l.points.size();
        if (P == 0) continue;
        l.velocity.resize(P, CartesianCoord{0.0, 0.0, 0.0});  // :88-90
        l.temperature.resize(P, 0.0);
        l.salinity.resize(P, 0.0);
        keep.push_back(&l);
        off.push_back(off.back() + (int64_t)P);
    }
    const int64_t m = (int64_t)keep.size(), T = off.back();
    std::vector<TrajectoryLine> out;
    out.reserve((size_t)m);
    if (m == 0) return out;
    std::vector<double> hp((size_t)T * 3), hv((size_t)T * 3), ht((size_t)T), hs((size_t)T), hl((size_t)m * 3);
    for (int64_t i = 0; i < m; ++i) {
        const TrajectoryLine& l = *keep[(size_t)i];
        const size_t P = l.points.size(), b = (size_t)off[(size_t)i];
        std::memcpy(hp.data() + 3 * b, l.points.data(), P * sizeof(CartesianCoord));
        std::memcpy(hv.data() + 3 * b, l.velocity.data(), P * sizeof(CartesianCoord));
        std::memcpy(ht.data() + b, l.temperature.data(), P * sizeof(double));
        std::memcpy(hs.data() + b, l.salinity.data(), P * sizeof(double));
    }
    // one allocation: points | velocity | temperature | salinity | last | offsets
    const size_t bytes = (size_t)T * 64 + (size_t)m * 24 + (size_t)(m + 1) * 8;
    struct DevBuf {
        void* p = nullptr;
        ~DevBuf() { (void)hipFree(p); }
    } buf;
    auto hip = [](hipError_t e, const char* what) {
        if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
    };
    hip(hipMalloc(&buf.p, bytes), "RemoveNaNTrajectoriesAndReindex: hipMalloc");
    double* dp = static_cast<double*>(buf.p);
    double* dv = dp + 3 * T;
    double* dt = dv + 3 * T;
    double* ds = dt + T;
    double* dl = ds + T;
    int64_t* doff = reinterpret_cast<int64_t*>(dl + 3 * m);
    const hipMemcpyKind h2d = hipMemcpyHostToDevice, d2h = hipMemcpyDeviceToHost;
    hip(hipMemcpy(dp, hp.data(), (size_t)T * 24, h2d), "hipMemcpy points");
    hip(hipMemcpy(dv, hv.data(), (size_t)T * 24, h2d), "hipMemcpy velocity");
    hip(hipMemcpy(dt, ht.data(), (size_t)T * 8, h2d), "hipMemcpy temperature");
    hip(hipMemcpy(ds, hs.data(), (size_t)T * 8, h2d), "hipMemcpy salinity");
    hip(hipMemcpy(doff, off.data(), (size_t)(m + 1) * 8, h2d), "hipMemcpy offsets");
    check(mops_remove_nan_ragged(m, doff, dp, dv, dt, ds, dl, nullptr), "mops_remove_nan_ragged");
    hip(hipMemcpy(hp.data(), dp, (size_t)T * 24, d2h), "hipMemcpy points");
    hip(hipMemcpy(hv.data(), dv, (size_t)T * 24, d2h), "hipMemcpy velocity");
    hip(hipMemcpy(ht.data(), dt, (size_t)T * 8, d2h), "hipMemcpy temperature");
    hip(hipMemcpy(hs.data(), ds, (size_t)T * 8, d2h), "hipMemcpy salinity");
    hip(hipMemcpy(hl.data(), dl, (size_t)m * 24, d2h), "hipMemcpy lastPoint");
    for (int64_t i = 0; i < m; ++i) {
        TrajectoryLine& l = *keep[(size_t)i];
        const size_t P = l.points.size(), b = (size_t)off[(size_t)i];
        std::memcpy(l.points.data(), hp.data() + 3 * b, P * sizeof(CartesianCoord));
        std::memcpy(l.velocity.data(), hv.data() + 3 * b, P * sizeof(CartesianCoord));
        std::memcpy(l.temperature.data(), ht.data() + b, P * sizeof(double));
        std::memcpy(l.salinity.data(), hs.data() + b, P * sizeof(double));
        l.lastPoint = {hl[(size_t)(3 * i)], hl[(size_t)(3 * i + 1)], hl[(size_t)(3 * i + 2)]};  // :123
        l.lineID = (int)i;  // :124
        out.push_back(l);
    }
    return out;
}

}  // namespace MOPS
