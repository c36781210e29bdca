// MOPS.h -- C++ operator API of the MI355X trajectory engine.
//
// Source-compatible mirror of the reference's public API for the trajectory
// path (YosefQiu/MOPS include/api/MOPS.h:20-148, settings structs
// src/Core/MPASOVisualizer.h:44-103, data model setters
// src/Core/MPASOGrid.cpp:82-188, src/Core/MPASOSolution.cpp:1145-1210):
// same names, argument meaning and error behaviour, implemented on the C ABI
// (include/mops_traj.h) -- the GPU engine is the only backend.
//
// Differences a caller can observe:
//   * vec3 is a plain {x, y, z} struct; the reference's backends rewrite
//     p.x() into p.x with a macro (BackendCompat.hpp:188-191) -- define
//     MOPS_COMPAT_ACCESSOR_MACROS before including this header to get the
//     same macros;
//   * MOPS_RunRemapping / regridding (image remapping) are out of scope and
//     return an empty result with an error message;
//   * derived fields are computed on the GPU and kept in HBM; nothing is
//     cached on disk (the reference's cache is keyed only by timestep, Q11).
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "mops_traj.h"

struct vec2 { double x, y; };
struct vec3 { double x, y, z; };
struct vec2i { int x, y; };
using SphericalCoord = vec2;
using CartesianCoord = vec3;

#ifdef MOPS_COMPAT_ACCESSOR_MACROS
#define x() x
#define y() y
#define z() z
#endif

namespace MOPS {

enum class CalcDirection : int { kForward, kBackward, kCount };
enum class CalcMethodType : int { kRK4, kEuler, kCount };
enum class GridAttributeType : int {
    kCellSize, kEdgeSize, kVertexSize, kMaxEdgesSize, kVertLevels, kVertLevelsP1, kVertexCoord, kCellCoord,
    kEdgeCoord, kVertexLatLon, kVerticesOnCell, kVerticesOnEdge, kCellsOnVertex, kCellsOnCell,
    kNumberVertexOnCell, kCellsOnEdge, kEdgesOnCell, kCellWeight, krefBottomDepth, kCount
};
enum class AttributeType : int {
    kZonalVelocity, kMeridionalVelocity, kVelocity, kNormalVelocity, kZTop, kLayerThickness, kBottomDepth, kCount
};

#define ONE_SECOND 1
#define ONE_MINUTE 60
#define ONE_HOUR 60 * 60
#define ONE_DAY 60 * 60 * 24
#define ONE_MONTH 60 * 60 * 24 * 30
#define ONE_YEAR 60 * 60 * 24 * 30 * 12

struct TrajectoryLine {
    int lineID;
    std::vector<CartesianCoord> points;
    std::vector<CartesianCoord> velocity;
    std::vector<double> temperature;
    std::vector<double> salinity;
    CartesianCoord lastPoint;
    double duration;
    double timestamp;
    double depth;
};

struct TrajectorySettings {
    size_t deltaT;
    size_t simulationDuration;
    size_t recordT;
    float depth;
    std::vector<float> particle_depths;
    std::string fileName;
    CalcDirection directionType = CalcDirection::kForward;
    CalcMethodType methodType = CalcMethodType::kEuler;
    bool hasPerParticleDepths() const { return !particle_depths.empty(); }
};

struct SamplingSettings {
    void setSampleRange(const vec2i& n) { sampleRange = n; }
    void setGeoBox(const vec2& lat, const vec2& lon) { sampleLatitudeRange = lat; sampleLongitudeRange = lon; }
    void setDepth(double d) { sampleDepth = d; }
    void setSamplingRegion(const vec2i& n, const vec2& lat, const vec2& lon, double d) {
        sampleRange = n; sampleLatitudeRange = lat; sampleLongitudeRange = lon; sampleDepth = d;
    }
    void atCellCenter(bool b) { bAtCellCenter = b; }
    vec2i getSampleRange() const { return sampleRange; }
    vec2 getLatitudeRange() const { return sampleLatitudeRange; }
    vec2 getLongitudeRange() const { return sampleLongitudeRange; }
    bool isAtCellCenter() const { return bAtCellCenter; }
    double getDepth() const { return sampleDepth; }

  private:
    vec2i sampleRange{0, 0};
    vec2 sampleLatitudeRange{0, 0};
    vec2 sampleLongitudeRange{0, 0};
    double sampleDepth = 0.0;
    bool bAtCellCenter = false;
};

// MPASOGrid: the members the trajectory path reads (MPASOGrid.h), 1-based size_t connectivity.
class MPASOGrid {
  public:
    void setGridAttribute(GridAttributeType type, int val);
    void setGridAttributesVec3(GridAttributeType type, const std::vector<vec3>& vec);
    void setGridAttributesVec2(GridAttributeType type, const std::vector<vec2>& vec);
    void setGridAttributesInt(GridAttributeType type, const std::vector<size_t>& vec);
    void setGridAttributesFloat(GridAttributeType type, const std::vector<float>& vec);
    bool checkAttribute() const;

    int mCellsSize = 0, mEdgesSize = 0, mMaxEdgesSize = 0, mVertexSize = 0, mVertLevels = 0, mVertLevelsP1 = 0;
    std::vector<vec3> vertexCoord_vec, cellCoord_vec, edgeCoord_vec;
    std::vector<vec2> vertexLatLon_vec;
    std::vector<size_t> verticesOnCell_vec, verticesOnEdge_vec, cellsOnVertex_vec, cellsOnCell_vec,
        numberVertexOnCell_vec, cellsOnEdge_vec, edgesOnCell_vec;
    std::vector<float> cellWeight_vec;
    std::string mCachedDataDir;
};

// SolutionID (MPASOSolution.h:12-16); timestep is value-initialised here
struct SolutionID {
    std::string timeStamp;
    int timestep = 0;
};

// MPASOSolution: raw per-cell fields of one snapshot (MPASOSolution.h).
class MPASOSolution {
  public:
    void setAttribute(GridAttributeType type, int val);
    void setAttributesDouble(AttributeType type, const std::vector<double>& vec);
    void setAttributesVec3(AttributeType type, const std::vector<vec3>& vec);
    void setTimestep(int t) { mTimesteps = t; }  // like the reference, does not touch mID
    // 32-bit FNV-1a of "<timeStamp>_<timestep>" (MPASOSolution.h:74-86)
    int getID() const {
        const std::string key = mID.timeStamp + "_" + std::to_string(mID.timestep);
        uint32_t h = 2166136261u;
        for (unsigned char c : key) h = (h ^ c) * 16777619u;
        return static_cast<int>(h);
    }
    std::string getTimeStamp() const { return mTimeStamp; }
    bool checkAttribute() const;

    int mCellsSize = 0, mEdgesSize = 0, mMaxEdgesSize = 0, mVertexSize = 0, mTimesteps = 0, mVertLevels = 0,
        mVertLevelsP1 = 0;
    SolutionID mID;
    std::string mTimeStamp;
    std::vector<double> cellLayerThickness_vec, cellBottomDepth_vec, cellSurfaceHeight_vec, cellZTop_vec,
        cellZonalVelocity_vec, cellMeridionalVelocity_vec, cellVertVelocity_vec, cellNormalVelocity_vec;
    std::vector<vec3> cellCenterVelocity_vec;
    std::map<std::string, std::vector<double>> mDoubleAttributes;
};

void MOPS_Init(const char* device = "gpu");
void MOPS_Begin();
void MOPS_AddGridMesh(std::shared_ptr<MPASOGrid> grid);
void MOPS_AddAttribute(int solID, std::shared_ptr<MPASOSolution> sol);
void MOPS_End();
void MOPS_ActiveAttribute(int t1, std::optional<int> t2 = std::nullopt);
std::vector<TrajectoryLine> MOPS_RunStreamLine(TrajectorySettings* config, std::vector<CartesianCoord>& sample_points);
std::vector<TrajectoryLine> MOPS_RunPathLine(TrajectorySettings* config, std::vector<CartesianCoord>& sample_points);
void MOPS_GenerateSamplePoints(SamplingSettings* config, std::vector<CartesianCoord>& sample_points);
// Extension (the reference has no teardown): releases the mesh and fields held in HBM by the
// global app.  Call it before the HIP runtime shuts down; nothing is freed from a static
// destructor at exit.
void MOPS_Finalize();

void MOPS_ResetTiming();
void MOPS_PrintTimingSummary();
void MOPS_PrintTimingDetailed();
double MOPS_GetCategoryTime(const char* category);
double MOPS_GetTotalTime();

// MPASOVisualizer::removeNaNTrajectoriesAndReindex (TrajectoryCommon.h:57-129), host form
std::vector<TrajectoryLine> RemoveNaNTrajectoriesAndReindex(std::vector<TrajectoryLine>& lines);

}  // namespace MOPS
