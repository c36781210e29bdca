/* mops_io.h -- trajectory output formats of the MI355X engine.
 *
 * Lines use the engine's dense layout (what mops_traj_finalize /
 * mops_run_trajectories produce): n lines of P points each,
 *   points, velocity  [n][P][3] f64 (x, y, z, metres / m s^-1)
 *   temperature, salinity [n][P] f64
 * The xyz -> geographic conversion runs on the GPU (mops_lines_geo); the
 * writers are host code streaming to a file, as the reference's are.
 */
#ifndef MOPS_IO_H
#define MOPS_IO_H

#include <stdint.h>

#include "mops_traj.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Per point {lat_deg, lon_deg, r, |v|}: GeoConverter::convertXYZToLatLonDegree
 * (src/Utils/GeoConverter.hpp:152-175: asin(z/r), atan2(y, x), x 180/pi),
 * r = sqrt(x*x + y*y + z*z) and the velocity magnitude the VTP writer stores
 * (VTKFileManager.hpp:389-395).  d_velocity may be NULL (|v| = 0).
 * Device buffers; d_geo is [n][P][4]. */
mops_status mops_lines_geo(int64_t n, int64_t P, const double* d_points, const double* d_velocity, double* d_geo,
                           void* stream);

/* VTKFileManager::SaveTrajectoryLinesAsVTP (src/IO/VTKFileManager.hpp:315-417):
 * one VTK XML PolyData file; points (lon, lat, 6371010 - r); a polyline per
 * trajectory, split where consecutive longitudes jump across +-170 deg;
 * point data "temperature", "salinity", "velocity_mag".  Lines with P == 0
 * are skipped.  h_geo from mops_lines_geo; temperature/salinity may be NULL
 * (NaN, as the reference's getTemp/getSal beyond the array).  `binary` != 0
 * writes appended raw little-endian data, 0 writes ASCII.  ".vtp" is appended
 * when missing (checkAndModifyExtension). */
mops_status mops_write_lines_vtp(const char* path, int64_t n, int64_t P, const double* h_geo,
                                 const double* h_temperature, const double* h_salinity, int binary);

/* The CLI's text dump (CLI/main.cpp:239-262): header line, then one line per
 * point "lineID point_idx px py pz vx vy vz" with std::ostream default
 * formatting. */
mops_status mops_write_lines_txt(const char* path, int64_t n, int64_t P, const double* h_points,
                                 const double* h_velocity);

/* export_pathlines_to_binary (tutorial/export_pathline_binary.py:27-125):
 * int32 particle count, then per particle int32 num_points and per point
 * lat, lon f64 [+ velocity_u, velocity_v, speed] [+ temperature, salinity],
 * little endian; plus "<path without suffix>.meta.json" with the field list
 * and per-particle byte offsets. */
mops_status mops_write_pathline_binary(const char* path, int64_t n, int64_t P, const double* h_geo,
                                       const double* h_velocity, const double* h_temperature,
                                       const double* h_salinity, int include_velocity, int include_scalars);

#ifdef __cplusplus
}
#endif
#endif /* MOPS_IO_H */
