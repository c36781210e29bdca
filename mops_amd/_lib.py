"""ctypes binding of the C ABI in include/mops_traj.h (libmops_traj.so).

This is the Python side of the drop-in boundary.  There is deliberately no
fallback: if the HIP library is missing the import of any engine entry point
raises, so a GPU box never silently runs something else.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmops_traj.so")

# every symbol include/mops_traj.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "mops_last_error", "mops_abi_version", "mops_selftest_math", "mops_selftest_walk",
    "mops_mesh_create", "mops_mesh_destroy", "mops_mesh_bytes", "mops_mesh_set_edges", "mops_cell_center_velocity_rbf",
    "mops_field_create", "mops_field_create_device", "mops_field_rebuild_device", "mops_field_create_derived", "mops_field_export", "mops_cell_to_vertex_attr",
    "mops_field_destroy", "mops_field_bytes",
    "mops_locate_cells", "mops_locate_cells_hinted", "mops_order_particles", "mops_order_scratch_bytes",
    "mops_order_particles_live", "mops_permute_arrays", "mops_records_clear_dead",
    "mops_traj_num_records", "mops_traj_num_steps", "mops_traj_advance", "mops_traj_finalize", "mops_traj_last_points",
    "mops_remove_nan_lines", "mops_remove_nan_ragged", "mops_run_trajectories", "mops_build_id",
    # include/mops_io.h
    "mops_lines_geo", "mops_write_lines_vtp", "mops_write_lines_txt", "mops_write_pathline_binary",
    # include/mops_netcdf.h
    "mops_nc_open", "mops_nc_close", "mops_nc_dim_len", "mops_nc_var_info", "mops_nc_read_f64", "mops_nc_read_i64",
    "mops_nc_read_bytes",
)

MOPS_OK, MOPS_ERR_INVALID, MOPS_ERR_HIP, MOPS_ERR_UNSUPPORTED = 0, -1, -2, -3
MOPS_FORWARD, MOPS_BACKWARD = 0, 1
MOPS_RK4, MOPS_EULER = 0, 1


class MeshDesc(C.Structure):
    _fields_ = [("n_cells", C.c_int64), ("n_vertices", C.c_int64), ("max_edges", C.c_int32),
                ("n_vert_levels", C.c_int32), ("h_n_edges_on_cell", C.c_void_p),
                ("h_vertices_on_cell", C.c_void_p), ("h_cells_on_cell", C.c_void_p),
                ("h_cells_on_vertex", C.c_void_p), ("h_cell_coord", C.c_void_p), ("h_vertex_coord", C.c_void_p)]


class SnapshotDesc(C.Structure):
    _fields_ = [("timestep", C.c_int32), ("h_layer_thickness", C.c_void_p), ("h_bottom_depth", C.c_void_p),
                ("h_surface_height", C.c_void_p), ("h_zonal_velocity", C.c_void_p),
                ("h_meridional_velocity", C.c_void_p), ("h_vert_velocity_top", C.c_void_p),
                ("h_normal_velocity", C.c_void_p)]


class TrajCfg(C.Structure):
    _fields_ = [("delta_t", C.c_int64), ("simulation_duration", C.c_int64), ("record_t", C.c_int64),
                ("direction", C.c_int32), ("method", C.c_int32)]


class Particles(C.Structure):
    _fields_ = [("n", C.c_int64), ("d_x", C.c_void_p), ("d_y", C.c_void_p), ("d_z", C.c_void_p),
                ("d_depth", C.c_void_p), ("d_cell", C.c_void_p), ("d_death_step", C.c_void_p),
                ("d_order", C.c_void_p), ("d_n_live", C.c_void_p)]


class PermArray(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("d_dst", C.c_void_p), ("elem_bytes", C.c_int64), ("rows", C.c_int64),
                ("row_stride", C.c_int64)]


class MopsError(RuntimeError):
    pass


_lib = None


def load(path: str | None = None):
    """Load libmops_traj.so; raise loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("MOPS_TRAJ_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise MopsError(f"HIP engine library not found at {path}: run `python -c \"import __graft_entry__ as g; "
                        f"g.build()\"` (hipcc --offload-arch=gfx950) first")
    # torch ships its own libamdhip64 (SONAME libamdhip64.so.7, but NEEDED as
    # "libamdhip64.so"): load it first so the engine binds to the same HIP
    # runtime instead of pulling a second copy from /opt/rocm -- two runtimes
    # in one process make the second one report "no ROCm-capable device".
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    P, I64, I32 = C.c_void_p, C.c_int64, C.c_int32
    st = C.c_int
    lib.mops_last_error.restype = C.c_char_p
    lib.mops_abi_version.restype = I32
    if os.path.abspath(path) == os.path.abspath(LIB_PATH):
        # the product library must be the build of the sources next to it (experiment variants
        # loaded through MOPS_TRAJ_LIB are exempt)
        from . import _build_id
        lib.mops_build_id.restype = C.c_char_p
        have = lib.mops_build_id().decode(errors="replace")
        want = _build_id.MARKER + _build_id.build_id()
        if have != want:
            raise MopsError(f"stale engine library {path}: built as {have!r}, the sources are {want!r}; rebuild with "
                            "`python -c \"import __graft_entry__ as g; g.build()\"`")
    lib.mops_build_id.restype = C.c_char_p
    if hasattr(lib, "mops_selftest_math"):  # (older engine builds timed as variants lack the self-test)
        lib.mops_selftest_math.argtypes = [I64, P, P, I32, P]; lib.mops_selftest_math.restype = st
    if hasattr(lib, "mops_selftest_walk"):
        lib.mops_selftest_walk.argtypes = [P, I64, P, P, P, P]; lib.mops_selftest_walk.restype = st
    lib.mops_mesh_create.argtypes = [P, P, P]; lib.mops_mesh_create.restype = st
    lib.mops_mesh_destroy.argtypes = [P]; lib.mops_mesh_destroy.restype = None
    lib.mops_mesh_bytes.argtypes = [P]; lib.mops_mesh_bytes.restype = I64
    lib.mops_mesh_set_edges.argtypes = [P, I64, P, P, P, P]; lib.mops_mesh_set_edges.restype = st
    lib.mops_cell_center_velocity_rbf.argtypes = [P, P, P, P]; lib.mops_cell_center_velocity_rbf.restype = st
    lib.mops_field_create.argtypes = [P, P, P, P]; lib.mops_field_create.restype = st
    lib.mops_field_create_device.argtypes = [P, P, P, P]; lib.mops_field_create_device.restype = st
    lib.mops_field_rebuild_device.argtypes = [P, P, P]; lib.mops_field_rebuild_device.restype = st
    lib.mops_field_create_derived.argtypes = [P, P, P, P, P, P]; lib.mops_field_create_derived.restype = st
    lib.mops_field_export.argtypes = [P, P, P, P, P]; lib.mops_field_export.restype = st
    lib.mops_cell_to_vertex_attr.argtypes = [P, P, P, P]; lib.mops_cell_to_vertex_attr.restype = st
    lib.mops_lines_geo.argtypes = [I64, I64, P, P, P, P]; lib.mops_lines_geo.restype = st
    lib.mops_write_lines_vtp.argtypes = [C.c_char_p, I64, I64, P, P, P, C.c_int]
    lib.mops_write_lines_vtp.restype = st
    lib.mops_write_lines_txt.argtypes = [C.c_char_p, I64, I64, P, P]; lib.mops_write_lines_txt.restype = st
    lib.mops_write_pathline_binary.argtypes = [C.c_char_p, I64, I64, P, P, P, P, C.c_int, C.c_int]
    lib.mops_write_pathline_binary.restype = st
    lib.mops_nc_open.argtypes = [C.c_char_p, P]; lib.mops_nc_open.restype = st
    lib.mops_nc_close.argtypes = [P]; lib.mops_nc_close.restype = None
    lib.mops_nc_dim_len.argtypes = [P, C.c_char_p, P]; lib.mops_nc_dim_len.restype = st
    lib.mops_nc_var_info.argtypes = [P, C.c_char_p, P, P, P, P]; lib.mops_nc_var_info.restype = st
    for fn in ("mops_nc_read_f64", "mops_nc_read_i64", "mops_nc_read_bytes"):
        getattr(lib, fn).argtypes = [P, C.c_char_p, I64, P, I64]
        getattr(lib, fn).restype = st
    lib.mops_field_destroy.argtypes = [P]; lib.mops_field_destroy.restype = None
    lib.mops_field_bytes.argtypes = [P]; lib.mops_field_bytes.restype = I64
    lib.mops_locate_cells.argtypes = [P, I64, P, P, P]; lib.mops_locate_cells.restype = st
    lib.mops_locate_cells_hinted.argtypes = [P, I64, P, P, P, P]; lib.mops_locate_cells_hinted.restype = st
    lib.mops_order_particles.argtypes = [P, I64, P, P, P]; lib.mops_order_particles.restype = st
    lib.mops_traj_num_records.argtypes = [P]; lib.mops_traj_num_records.restype = I64
    lib.mops_traj_num_steps.argtypes = [P]; lib.mops_traj_num_steps.restype = I64
    lib.mops_traj_advance.argtypes = [P, P, P, P, P, I64, I64, P, I64, P]; lib.mops_traj_advance.restype = st
    lib.mops_traj_finalize.argtypes = [I64, I64, P, P, I64, I32, P, P, P, P, P, P, P]
    lib.mops_traj_finalize.restype = st
    lib.mops_traj_last_points.argtypes = [I64, I64, P, P, I64, P, P, P]
    lib.mops_traj_last_points.restype = st
    lib.mops_remove_nan_lines.argtypes = [I64, I64, P, P, P, P, P, P]; lib.mops_remove_nan_lines.restype = st
    lib.mops_remove_nan_ragged.argtypes = [I64, P, P, P, P, P, P, P]; lib.mops_remove_nan_ragged.restype = st
    lib.mops_order_scratch_bytes.argtypes = [I64]; lib.mops_order_scratch_bytes.restype = I64
    lib.mops_permute_arrays.argtypes = [I64, P, I32, P, P]; lib.mops_permute_arrays.restype = st
    lib.mops_order_particles_live.argtypes = [P, I64, P, P, P, P, P, I64, P]
    lib.mops_order_particles_live.restype = st
    lib.mops_records_clear_dead.argtypes = [I64, P, I64, I64, P, I64, P]
    lib.mops_records_clear_dead.restype = st
    lib.mops_run_trajectories.argtypes = [P, P, P, P, I64, P, P, C.c_float, P, P, P, P, P, P, P, P, P, P]
    lib.mops_run_trajectories.restype = st
    _lib = lib
    return lib


def check(status: int, what: str = ""):
    if status != MOPS_OK:
        msg = load().mops_last_error().decode(errors="replace")
        raise MopsError(f"{what} failed (status {status}): {msg}")
