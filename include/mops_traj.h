/*
 * mops_traj.h -- C ABI of the MI355X (gfx950) particle-trajectory engine.
 *
 * Drop-in boundary for the reference's trajectory path (YosefQiu/MOPS):
 * every entry point below replaces one reference interface, cited per
 * function.  Plain pointers and sizes only; no C++ or torch types.  Device
 * pointers are named d_*, host pointers h_*; `stream` is a hipStream_t
 * passed as void* (NULL = the default stream).
 *
 * Conventions taken from the reference so a caller can pass its own arrays
 * unchanged:
 *   - connectivity is size_t (uint64_t), 1-based, 0 = missing
 *     (MPASOGrid::verticesOnCell_vec / cellsOnCell_vec / cellsOnVertex_vec,
 *     src/Core/MPASOGrid.h);
 *   - coordinates are AoS xyz doubles (std::vector<vec3>::data());
 *   - fields are row-major [entity][level] (MPASOSolution vectors).
 * Internally the engine keeps its own int32 0-based, per-cell-record layout
 * in HBM.
 *
 * Error convention: every function returns mops_status.  MOPS_ERR_INVALID
 * is what the reference answers with Error() + an empty result
 * (MPASOVisualizerKernels.cpp:659-669); mops_last_error() gives the text.
 * Per-particle failures are not errors: the particle stops ("dies") exactly
 * where the reference's lambda returns, and its death step is reported.
 */
#ifndef MOPS_TRAJ_H
#define MOPS_TRAJ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    MOPS_OK = 0,
    MOPS_ERR_INVALID = -1,     /* bad arguments / settings (reference: Error() + {}) */
    MOPS_ERR_HIP = -2,         /* HIP runtime failure */
    MOPS_ERR_UNSUPPORTED = -3  /* e.g. maxEdges > 20 (reference MAX_VERTEX_NUM) */
} mops_status;

/* CalcDirection / CalcMethodType (src/Core/MPASOVisualizer.h:14-15) */
enum { MOPS_FORWARD = 0, MOPS_BACKWARD = 1 };
enum { MOPS_RK4 = 0, MOPS_EULER = 1 };

typedef struct mops_mesh mops_mesh;    /* device-resident mesh (opaque) */
typedef struct mops_field mops_field;  /* device-resident derived snapshot (opaque) */

/* Host description of an MPAS-O mesh, in MPASOGrid's storage form. */
typedef struct {
    int64_t n_cells;                     /* mCellsSize */
    int64_t n_vertices;                  /* mVertexSize */
    int32_t max_edges;                   /* mMaxEdgesSize */
    int32_t n_vert_levels;               /* mVertLevels (the w grid has +1) */
    const uint64_t* h_n_edges_on_cell;   /* numberVertexOnCell_vec [C] */
    const uint64_t* h_vertices_on_cell;  /* verticesOnCell_vec [C*maxE] */
    const uint64_t* h_cells_on_cell;     /* cellsOnCell_vec [C*maxE] */
    const uint64_t* h_cells_on_vertex;   /* cellsOnVertex_vec [V*3] */
    const double* h_cell_coord;          /* cellCoord_vec [C*3] */
    const double* h_vertex_coord;        /* vertexCoord_vec [V*3] */
} mops_mesh_desc;

/* Raw per-cell fields of one history snapshot (MPASOSolution members). */
typedef struct {
    int32_t timestep;                    /* mTimesteps (informational) */
    const double* h_layer_thickness;     /* cellLayerThickness_vec [C*L] (required) */
    const double* h_bottom_depth;        /* cellBottomDepth_vec [C] or NULL */
    const double* h_surface_height;      /* cellSurfaceHeight_vec [C] or NULL */
    const double* h_zonal_velocity;      /* cellZonalVelocity_vec [C*L] */
    const double* h_meridional_velocity; /* cellMeridionalVelocity_vec [C*L] */
    const double* h_vert_velocity_top;   /* cellVertVelocity_vec [C*(L+1)] or NULL (= 0) */
    const double* h_normal_velocity;     /* cellNormalVelocity_vec [E*L] or NULL: used only when the
                                            zonal/meridional pair is absent, on a mesh with edges
                                            (mops_mesh_set_edges) -- the RBF reconstruction */
} mops_snapshot_desc;

/* TrajectorySettings (src/Core/MPASOVisualizer.h:90-103); seconds. */
typedef struct {
    int64_t delta_t;                     /* deltaT */
    int64_t simulation_duration;         /* simulationDuration */
    int64_t record_t;                    /* recordT */
    int32_t direction;                   /* MOPS_FORWARD / MOPS_BACKWARD */
    int32_t method;                      /* MOPS_RK4 / MOPS_EULER (reference default Euler) */
} mops_traj_cfg;

/* Device-resident particle state, SoA, caller-owned (n entries each). */
typedef struct {
    int64_t n;
    double* d_x;                         /* stable_points x,y,z (updated in place) */
    double* d_y;
    double* d_z;
    float* d_depth;                      /* effective_depths (float, as the reference) */
    int32_t* d_cell;                     /* in: seed cell (default_cell_id), then current cell */
    int32_t* d_death_step;               /* out: -1 alive, else the step it died at */
    const int32_t* d_order;              /* optional processing order (slot -> particle index),
                                            from mops_order_particles; NULL = identity.  Only
                                            affects speed, never results. */
    const int32_t* d_n_live;             /* optional device count: only slots [0, *d_n_live) hold
                                            live particles (after mops_order_particles_live); the
                                            launch spreads just those over the XCDs.  NULL = all n. */
} mops_particles;

const char* mops_last_error(void);
int32_t mops_abi_version(void);

/* Self-test of the trajectory kernel's exact math helpers on the device (not
 * a reference entry point): for n doubles at d_x, op 0 writes {fast sqrt,
 * sqrt()} pairs, op 1 writes {fast sin, sin(), fast cos, cos()} (|x| < 0.78
 * only; other x copy the library values) into d_out (2n or 4n doubles); op 2
 * reads n 3-vectors (3n doubles) and writes {fast a_j / |a| (j = 0..2), a_j / |a|}
 * (6n doubles; zeros where |a| <= 1e-12). */
mops_status mops_selftest_math(int64_t n, const double* d_x, double* d_out, int32_t op, void* stream);

/* Self-test of the trajectory kernel's exact neighbour-table shortcut (not a
 * reference entry point; maxEdges <= 7 meshes): for n points d_pts [n][3] in
 * cells d_cells [n], d_out [n] gets bit 0 = the float bisector test kept the
 * cell, bit 1 = the one-hop walk (MPASOVisualizerKernels.cpp:902-922) kept it,
 * bits 8.. = the stay radius the test set (metres); -1 for an invalid cell.
 * Bit 0 without bit 1 would be a wrong shortcut. */
mops_status mops_selftest_walk(const mops_mesh* mesh, int64_t n, const double* d_pts, const int32_t* d_cells,
                               int32_t* d_out, void* stream);

/* ---- mesh / snapshots -------------------------------------------------- */

/* Upload + re-layout a mesh.  Replaces MOPSApp::addGrid / MPASOGrid
 * (src/Core/MOPSApp.cpp:65-75): the KD-tree build becomes the engine's
 * bucket index for mops_locate_cells. */
mops_status mops_mesh_create(const mops_mesh_desc* desc, void* stream, mops_mesh** out);
void mops_mesh_destroy(mops_mesh* mesh);
/* Bytes the mesh occupies in HBM. */
int64_t mops_mesh_bytes(const mops_mesh* mesh);

/* Upload the mesh's edges (MPASOGrid edgesOnCell_vec [C*maxE], cellsOnEdge_vec
 * [E*2], edgeCoord_vec [E*3], reference storage form) for the RBF
 * reconstruction of the cell-centre velocity from edge-normal velocities
 * (TBBBackend::CalcCellCenterVelocity, src/CPU/TBB/MPASOSolutionTBB.cpp:131-245,
 * reached through MPASOSolution::calcCellCenterVelocity,
 * src/Core/MPASOSolution.cpp:85-110).  The per-cell RBF systems depend on the
 * geometry only and are solved here once.  MOPS_ERR_UNSUPPORTED if a cell has
 * more than 7 edges (the reference's stencil arrays hold MAX_VERTEX_NUM = 7). */
mops_status mops_mesh_set_edges(mops_mesh* mesh, int64_t n_edges, const uint64_t* h_edges_on_cell,
                                const uint64_t* h_cells_on_edge, const double* h_edge_coord, void* stream);
/* The RBF cell-centre velocity [C*L*3] from the edge-normal velocity [E*L]
 * (device pointers) -- TBBBackend::CalcCellCenterVelocity's output, bit for
 * bit, quirks included: the stencil always has 7 points (absent edges enter
 * as zero points with zero unit vectors, which makes the 7x7 system singular,
 * i.e. NaN, for every cell with fewer than 7 edges), alpha is 1 and the
 * right-hand side evaluates the RBF at 1 (Interpolation.hpp:223-302). */
mops_status mops_cell_center_velocity_rbf(const mops_mesh* mesh, const double* d_normal_velocity, double* d_out,
                                          void* stream);

/* Upload raw fields and derive, on the GPU, the vertex arrays the trajectory
 * kernels read.  Replaces MOPSApp::addSol's preprocessing chain
 * (src/Core/MOPSApp.cpp:100-129): MPASOSolution::calcCellCenterZtop
 * (MPASOSolution.cpp:535-618), TBBBackend::CalcCellVertexZtop
 * (MPASOSolutionTBB.cpp:9-55), CalcCellCenterVelocityByZM (:108-129) -- or,
 * for a snapshot with edge normals only, CalcCellCenterVelocity (:131-245),
 * CalcCellVertexVelocity (:270-318), CalcCellVertexVertVelocity (:320-366). */
mops_status mops_field_create(const mops_mesh* mesh, const mops_snapshot_desc* desc, void* stream,
                              mops_field** out);
/* As mops_field_create, but every array pointer in d_desc is a DEVICE pointer
 * (raw fields already in HBM, e.g. decoded or generated on the GPU); they are
 * read in place and stay owned by the caller.  Same preprocessing chain
 * (MOPSApp::addSol, src/Core/MOPSApp.cpp:100-129); lets a snapshot-chaining
 * driver (tutorial/pathLine.cpp:244-309) stream snapshots without a host
 * round trip. */
mops_status mops_field_create_device(const mops_mesh* mesh, const mops_snapshot_desc* d_desc, void* stream,
                                     mops_field** out);
/* Re-derive a field made by mops_field_create_device from another snapshot's
 * raw DEVICE arrays, in place: no allocation, asynchronous on `stream`.  The
 * reference rebuilds MPASOSolution per snapshot (MOPSApp::addSol); here a
 * pair-chaining driver recycles the buffers of the snapshot it just finished
 * (stream order: every earlier trajectory launch reading `field` on `stream`
 * completes first).  The raw arrays must stay valid until the work runs. */
mops_status mops_field_rebuild_device(mops_field* field, const mops_snapshot_desc* d_desc, void* stream);
/* Upload already-derived vertex arrays (cellVertexZTop_vec [V*L],
 * cellVertexVelocity_vec [V*L*3], cellVertexVertVelocity_vec [V*(L+1)]);
 * the path MOPSApp::addSol takes when they are pre-set (MOPSApp.cpp:100,107,117). */
mops_status mops_field_create_derived(const mops_mesh* mesh, const double* h_vertex_ztop,
                                      const double* h_vertex_vel, const double* h_vertex_w,
                                      void* stream, mops_field** out);
/* Copy the derived vertex arrays back to the host (any pointer may be NULL). */
mops_status mops_field_export(const mops_field* field, double* h_vertex_ztop, double* h_vertex_vel,
                              double* h_vertex_w, void* stream);
/* CalcCellCenterToVertex (MPASOSolutionTBB.cpp:57-106) for one double
 * attribute [C*L] -> [V*L] (negative results clamped to 0), device pointers. */
mops_status mops_cell_to_vertex_attr(const mops_mesh* mesh, const double* d_cell_attr, double* d_vertex_attr,
                                     void* stream);
void mops_field_destroy(mops_field* field);
int64_t mops_field_bytes(const mops_field* field);

/* ---- seed location ----------------------------------------------------- */

/* Exact nearest cell centre (Euclidean) for n points [n*3] (device
 * pointers).  Replaces MPASOField::calcInWhichCells -> MPASOGrid::searchKDT
 * (src/Core/MPASOField.cpp:23-34, src/Core/MPASOGrid.cpp:287-313, nanoflann
 * 1-NN).  Ties resolve to the smallest cell index. */
mops_status mops_locate_cells(const mops_mesh* mesh, int64_t n, const double* d_points, int32_t* d_cells,
                              void* stream);

/* Same answer as mops_locate_cells, faster when a candidate cell per point is
 * known (d_hint [n], device, may be NULL; entries outside [0, C) are
 * ignored): a point within half the distance from its hint's centre to the
 * nearest OTHER centre (less 1 m) provably has the hint as its unique nearest
 * centre, and skips the search.  Used between chained pathline pairs, where
 * each continuation point's hint is the cell its particle ended in
 * (pyMOPSAPI.py:1446-1459 re-locates every pair's seeds). */
mops_status mops_locate_cells_hinted(const mops_mesh* mesh, int64_t n, const double* d_points,
                                     const int32_t* d_hint, int32_t* d_cells, void* stream);

/* Locality order for n particles: sorts particle indices by a Morton key
 * of their current cell centre, so a wavefront's lanes share cell stencils
 * (no reference counterpart: the reference processes particles in index
 * order).  d_cell [n] -> d_order [n] (device). */
mops_status mops_order_particles(const mops_mesh* mesh, int64_t n, const int32_t* d_cell, int32_t* d_order,
                                 void* stream);

/* Out-of-place gather of particle arrays by a slot order, all in one launch
 * (no reference counterpart: the locality order is the engine's own):
 * dst[row][i] = src[row][d_order[i]] for i < n (d_order NULL = copy), for up
 * to 16 arrays of 4-, 8- or 24-byte elements, each with `rows` rows
 * `row_stride` elements apart (e.g. the [K][6][stride] record slab). */
typedef struct {
    const void* d_src;
    void* d_dst;                         /* must differ from d_src */
    int64_t elem_bytes;                  /* 4, 8 or 24 */
    int64_t rows;                        /* >= 1 */
    int64_t row_stride;                  /* elements between rows (>= n when rows > 1) */
} mops_perm_array;
mops_status mops_permute_arrays(int64_t n, const int32_t* d_order, int32_t count, const mops_perm_array* arrays,
                                void* stream);

/* Dead-particle compaction (no reference counterpart: the reference's
 * parallel_for keeps visiting particles whose lambda has returned,
 * MPASOVisualizerKernels.cpp:944-957, quirk Q1).  As mops_order_particles,
 * but particles with d_death[i] >= 0 (d_death may be NULL) sort after every
 * live one, so live particles fill whole waves; d_n_live (device, may be
 * NULL) receives their count, for mops_particles::d_n_live.  Re-entrant: the caller passes device scratch of
 * at least mops_order_scratch_bytes(n) bytes, so several particle parts can
 * be re-sorted concurrently on their own streams. */
int64_t mops_order_scratch_bytes(int64_t n);
mops_status mops_order_particles_live(const mops_mesh* mesh, int64_t n, const int32_t* d_cell,
                                      const int32_t* d_death, int32_t* d_order, int32_t* d_n_live,
                                      void* d_scratch, int64_t scratch_bytes, void* stream);
/* Zero record slots [k_begin, K) of slots [*d_n_live, n) (d_records [K][6][record_stride]):
 * after a compaction that moved only the sampled slots [0, k_begin), the dead particles now
 * at the end carry the zeros of their unsampled slots again (see mops_traj_advance).  No
 * reference counterpart (the reference never re-sorts). */
mops_status mops_records_clear_dead(int64_t n, const int32_t* d_n_live, int64_t k_begin, int64_t K,
                                    double* d_records, int64_t record_stride, void* stream);

/* ---- trajectory hot path (device-resident) ----------------------------- */

/* Number of record slots K = simulation_duration / record_t (reference
 * each_points_size, MPASOVisualizerKernels.cpp:703). */
int64_t mops_traj_num_records(const mops_traj_cfg* cfg);
/* Number of integration steps = simulation_duration / delta_t. */
int64_t mops_traj_num_steps(const mops_traj_cfg* cfg);

/* Advance particles over global steps [step_begin, step_end) of one
 * StreamLine (back == NULL; Kernel::StreamLine, MPASOVisualizerKernels.cpp:
 * 874-1003) or PathLine (Kernel::PathLine, :1329-1483) call.  Records go to
 * d_records laid out [K][6][record_stride] doubles (px,py,pz,vx,vy,vz);
 * slot 0 also receives the seed / first-step velocity pre-writes
 * (:901, :990).  d_records needs no initialisation when the calls start at
 * step 0: every slot a particle does not sample (after its death, past the
 * run's last record step, or all of them for a particle already dead at step
 * 0) is written with the zeros of the reference's vector::resize zero-init --
 * at its death or by the call that reaches n_steps.  A caller whose
 * first call starts after step 0 passes records zero-filled.  Calling it over
 * consecutive step ranges is identical to one call over [0, n_steps); a
 * caller that moves particles between slots in between (a re-sort) moves
 * every record slot, or clears the moved dead particles' unsampled slots
 * (mops_records_clear_dead).
 * Streams: pathline launches keep one small device flag per HIP stream in
 * the mesh (the cooperative-tile selection), freed with the mesh.  Use
 * long-lived streams (torch's pool, or streams created once): a stream
 * destroyed while its launches still run, whose handle a new stream then
 * reuses, would share that flag with the old launches. */
mops_status mops_traj_advance(const mops_mesh* mesh, const mops_field* front, const mops_field* back,
                              const mops_traj_cfg* cfg, const mops_particles* particles,
                              int64_t step_begin, int64_t step_end, double* d_records,
                              int64_t record_stride, void* stream);

/* FinalizeTrajectoryLines[WithAttrs] + RemoveNaNTrajectoriesAndReindex
 * (src/Common/TrajectoryCommon.h:57-190) on the device: seeds [n*3] and
 * records -> points/velocity [n*(K+1)*3], temperature/salinity [n*(K+1)]
 * (pathline: velocity x/y, reference quirk Q9; streamline: zeros),
 * last point [n*3].  d_line [n] (or NULL = identity) maps particle slot i of
 * seeds/records to output line d_line[i] -- for particles kept physically in
 * locality order (the record stores of mops_traj_advance then coalesce).
 * Any output pointer except points may be NULL. */
mops_status mops_traj_finalize(int64_t n, int64_t K, const double* d_seeds, const double* d_records,
                               int64_t record_stride, int32_t pathline, const int32_t* d_line, double* d_points,
                               double* d_velocity, double* d_temperature, double* d_salinity, double* d_last_point,
                               void* stream);

/* mops_traj_finalize's d_last_point alone: each line's cleaned last point
 * (RemoveNaNTrajectoriesAndReindex, src/Common/TrajectoryCommon.h:92-121:
 * the last finite point before the first non-finite one) from the seeds and
 * the records' positions, written at d_line[i] (NULL = identity).  What the
 * next pair of a chain needs as its seeds (MOPSPathline.run's _last_pt,
 * tutorial/pyMOPSAPI.py:1488), so the full line assembly can run
 * beside the next pair.  Same values as mops_traj_finalize's bit for bit. */
mops_status mops_traj_last_points(int64_t n, int64_t K, const double* d_seeds, const double* d_records,
                                  int64_t record_stride, const int32_t* d_line, double* d_last_point, void* stream);

/* RemoveNaNTrajectoriesAndReindex alone on n lines of P points each, in
 * place (device pointers; [n*P*3], [n*P*3], [n*P], [n*P], out [n*3]). */
mops_status mops_remove_nan_lines(int64_t n, int64_t P, double* d_points, double* d_velocity,
                                  double* d_temperature, double* d_salinity, double* d_last_point, void* stream);
/* The same for ragged lines -- the reference's vector<TrajectoryLine>, whose
 * lines may differ in length (RemoveNaNTrajectoriesAndReindex,
 * src/Common/TrajectoryCommon.h:57-129; test/test_trajector.cpp:26-194):
 * line i is points [d_offsets[i], d_offsets[i+1]) of the packed arrays
 * (d_offsets [n+1], device), velocity/temperature/salinity already resized to
 * the points' length (:88-90).  One launch for all lines; an empty line is
 * left untouched (the reference drops it and re-indexes the rest, which is
 * host bookkeeping).  d_last_point [n*3] gets each non-empty line's last point. */
mops_status mops_remove_nan_ragged(int64_t n, const int64_t* d_offsets, double* d_points, double* d_velocity,
                                   double* d_temperature, double* d_salinity, double* d_last_point, void* stream);

/* Identity of the engine build: a hash of the engine's sources, headers,
 * compiler flags and ROCm version, stamped at compile time (no reference
 * counterpart).  The Python loader refuses a library whose id differs from
 * the sources next to it, so a stale binary never runs. */
const char* mops_build_id(void);

/* ---- host convenience (the backend plug point) ------------------------- */

/* MOPS::Factory::StreamLine / PathLine (src/Common/MOPSFactory.h:27-39)
 * with host buffers: seeds [n*3]; depths [n] or NULL (then `depth` for all,
 * BuildEffectiveDepths, TrajectoryCommon.h:29-41); cells [n] in/out or NULL
 * (entries < 0 are located, as default_cell_id); outputs as
 * mops_traj_finalize plus the final positions (the caller's
 * sample_points update in MOPSApp::runPathLine, MOPSApp.cpp:287-290) and
 * death steps.  Any output pointer except h_points may be NULL. */
mops_status mops_run_trajectories(const mops_mesh* mesh, const mops_field* front, const mops_field* back,
                                  const mops_traj_cfg* cfg, int64_t n, const double* h_seeds,
                                  const float* h_depths, float depth, int32_t* h_cells, double* h_points,
                                  double* h_velocity, double* h_temperature, double* h_salinity,
                                  double* h_last_point, double* h_final_pos, float* h_final_depth,
                                  int32_t* h_death_step, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MOPS_TRAJ_H */
