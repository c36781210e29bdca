/* mops_netcdf.h -- native reader for MPAS netCDF files in the classic
 * formats (CDF-1, CDF-2 "64-bit offset", CDF-5 "64-bit data"), replacing the
 * netCDF-C / ftk::ndarray calls of the reference's MPASOReader
 * (src/IO/MPASOReader.cpp:96-245) for the arrays the trajectory path needs
 * (SURVEY §8 f2).  netCDF-4/HDF5 files are rejected with MOPS_ERR_UNSUPPORTED.
 *
 * Variables are read whole (non-record) or one record at a time (variables
 * whose first dimension is the unlimited "Time"), converted to f64 / i64 /
 * bytes, in the file's row-major order.
 */
#ifndef MOPS_NETCDF_H
#define MOPS_NETCDF_H

#include <stdint.h>

#include "mops_traj.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mops_nc mops_nc;

/* netCDF external types (NC_BYTE .. NC_UINT64) */
enum { MOPS_NC_BYTE = 1, MOPS_NC_CHAR, MOPS_NC_SHORT, MOPS_NC_INT, MOPS_NC_FLOAT, MOPS_NC_DOUBLE, MOPS_NC_UBYTE,
       MOPS_NC_USHORT, MOPS_NC_UINT, MOPS_NC_INT64, MOPS_NC_UINT64 };

/* nc_open(NC_NOWRITE): parse the header. */
mops_status mops_nc_open(const char* path, mops_nc** out);
void mops_nc_close(mops_nc* nc);

/* nc_inq_dimid + nc_inq_dimlen; the unlimited dimension reports the record
 * count.  MOPS_ERR_INVALID if absent. */
mops_status mops_nc_dim_len(const mops_nc* nc, const char* name, int64_t* len);

/* Variable metadata: external type, rank, shape (up to 8 dims; the record
 * dimension reports the record count) and whether it is a record variable.
 * MOPS_ERR_INVALID if absent. */
mops_status mops_nc_var_info(const mops_nc* nc, const char* name, int32_t* type, int32_t* ndims, int64_t* shape,
                             int32_t* is_record);

/* Read a variable converted to f64 (numeric types) / i64 (integer types) /
 * raw bytes (NC_CHAR, NC_BYTE, NC_UBYTE).  For a record variable `record`
 * selects one record and `count` must be the product of the remaining
 * dimensions; for other variables `record` must be 0 and `count` the total
 * size. */
mops_status mops_nc_read_f64(const mops_nc* nc, const char* name, int64_t record, double* out, int64_t count);
mops_status mops_nc_read_i64(const mops_nc* nc, const char* name, int64_t record, int64_t* out, int64_t count);
mops_status mops_nc_read_bytes(const mops_nc* nc, const char* name, int64_t record, char* out, int64_t count);

#ifdef __cplusplus
}
#endif
#endif /* MOPS_NETCDF_H */
