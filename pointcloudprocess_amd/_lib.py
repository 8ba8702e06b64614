"""ctypes binding of libpcp.so (the HIP/gfx950 implementation behind include/pcp.h).

The product path has no CPU fallback: if the in-tree library is missing or cannot be
loaded, importing the ops raises immediately.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# A/B measurements only: PCP_LIB names another build of the library, and is honoured only together
# with PCP_AB=1 (tools/*_ab.sh set both); the product and the tests always load the in-tree build
_AB = os.environ.get("PCP_AB") == "1" and bool(os.environ.get("PCP_LIB"))
LIB_PATH = os.environ["PCP_LIB"] if _AB else os.path.join(HERE, "libpcp.so")

PCP_OK = 0
_STATUS = {
    -1: "PCP_ERR_ARG", -2: "PCP_ERR_HIP", -3: "PCP_ERR_NOMEM", -4: "PCP_ERR_EMPTY",
    -5: "PCP_ERR_UNSUPPORTED", -6: "PCP_ERR_ICP", -7: "PCP_ERR_CAPACITY",
}

# every symbol declared in include/pcp.h: (name, restype, argtypes)
_vp, _i32, _i64, _sz, _f32, _f64, _u32 = (C.c_void_p, C.c_int, C.c_int64, C.c_size_t,
                                          C.c_float, C.c_double, C.c_uint32)
_P = C.POINTER
SIGNATURES = [
    ("pcp_abi_version", _i32, []),
    ("pcp_ctx_create", _i32, [_i32, _vp, _P(_vp)]),
    ("pcp_ctx_destroy", _i32, [_vp]),
    ("pcp_ctx_set_stream", _i32, [_vp, _vp]),
    ("pcp_ctx_stream", _vp, [_vp]),
    ("pcp_last_error", C.c_char_p, [_vp]),
    ("pcp_sync", _i32, [_vp]),
    ("pcp_malloc", _i32, [_vp, _P(_vp), _sz]),
    ("pcp_free", _i32, [_vp, _vp]),
    ("pcp_memcpy_h2d", _i32, [_vp, _vp, _vp, _sz]),
    ("pcp_memcpy_d2h", _i32, [_vp, _vp, _vp, _sz]),
    ("pcp_memset", _i32, [_vp, _vp, _i32, _sz]),
    ("pcp_index_build_f64", _i32, [_vp, _vp, _sz, _i64, _vp, _i64, _f64, _P(_vp)]),
    ("pcp_index_build_f32", _i32, [_vp, _vp, _sz, _i64, _f64, _P(_vp)]),
    ("pcp_index_destroy", _i32, [_vp]),
    ("pcp_index_size", _i64, [_vp]),
    ("pcp_index_identity_mapping", _i32, [_vp]),
    ("pcp_index_cell_size", _f64, [_vp]),
    ("pcp_index_cells", _i64, [_vp]),
    ("pcp_index_sorted_points", _vp, [_vp]),
    ("pcp_knn", _i32, [_vp, _vp, _vp, _sz, _i64, _i32, _vp, _vp]),
    ("pcp_radius_count", _i32, [_vp, _vp, _vp, _sz, _i64, _f64, _u32, _vp]),
    ("pcp_radius_fill", _i32, [_vp, _vp, _vp, _sz, _i64, _f64, _u32, _vp, _vp, _vp]),
    ("pcp_index_build_h16", _i32, [_vp, _vp, _sz, _i64, _f64, _P(_vp)]),
    ("pcp_h16_radius_count", _i32, [_vp, _vp, _f32, _i64, _vp]),
    ("pcp_h16_radius_fill", _i32, [_vp, _vp, _f32, _i64, _vp, _vp, _vp, _vp]),
    ("pcp_scan_counts", _i32, [_vp, _vp, _i64, _vp, _P(_i64)]),
    ("pcp_knn_bruteforce", _i32, [_vp, _vp, _sz, _i64, _vp, _sz, _i64, _i32, _vp, _vp]),
    ("pcp_knn_bruteforce_last_fallback", _i32, [_vp, _vp]),
    ("pcp_nearest_query", _i32, [_vp, _vp, _vp, _sz, _i64, _f64, _vp, _vp]),
    ("pcp_normals_rpca", _i32, [_vp, _vp, _sz, _i64, _vp, _i32, _f32, _f32, C.c_uint64, _vp]),
    ("pcp_plane_fit_segments", _i32, [_vp, _vp, _sz, _vp, _vp, _i64, _vp]),
    ("pcp_region_growing", _i32, [_vp, _vp, _vp, _sz, _i64, _vp, _f64, _f64, _vp, _vp, _vp, _P(_i64)]),
    ("pcp_knn_lod", _i32, [_vp, _vp, _i64, _vp, _i64, _i32, _vp, _vp]),
    ("pcp_minmax_aos48", _i32, [_vp, _vp, _i64, _i32, _P(_f64), _P(_f64)]),
    ("pcp_centroid_aos48", _i32, [_vp, _vp, _i64, _i32, _P(_f64), _P(_u32)]),
    ("pcp_centroid_concat_aos48", _i32, [_vp, _vp, _i64, _vp, _i64, _i32, _P(_f64), _P(_u32)]),
    ("pcp_transform_aos48", _i32, [_vp, _vp, _vp, _i64, _i32, _P(_f64)]),
    ("pcp_voxel_filter", _i32, [_vp, _vp, _i64, _i32, _P(_f64), _i32, _vp, _P(_i64), _vp]),
    ("pcp_pose_interpolate", _i32, [_vp, _i64, _i64, _i64]),
    ("pcp_pcd_write", _i32, [C.c_char_p, _vp, _i64, _i64, _i64, _i32]),
    ("pcp_pcd_read", _i32, [C.c_char_p, _vp, _i64, _P(_i64)]),
    ("pcp_pcd_read_ex", _i32, [C.c_char_p, _vp, _i64, _P(_i64), _P(_i64), _P(_i64), _P(_i32)]),
    ("pcp_lzf_compress", _sz, [_vp, _sz, _vp, _sz]),
    ("pcp_lzf_decompress", _sz, [_vp, _sz, _vp, _sz]),
    ("pcp_grid_create", _i32, [_vp, _P(_vp)]),
    ("pcp_grid_destroy", _i32, [_vp]),
    ("pcp_grid_clear", _i32, [_vp, _vp]),
    ("pcp_grid_add_cloud", _i32, [_vp, _vp, _vp, _i64]),
    ("pcp_grid_size", _i64, [_vp]),
    ("pcp_grid_cells", _i64, [_vp]),
    ("pcp_grid_points", _i32, [_vp, _vp, _vp, _i64, _P(_i64)]),
    ("pcp_grid_box", _i32, [_vp, _vp, _i32, _i32, _i32, _i32, _vp, _i64, _P(_i64)]),
    ("pcp_grid_match", _i32, [_vp, _vp, _vp, _i64, _f32, _vp, _P(_i64), _vp, _i64, _P(_i64)]),
    ("pcp_pose_lum_elch", _i32, [_vp, _i64, _i64, _i64, _vp]),
    ("pcp_pose_loop_closure", _i32, [_vp, _vp, _i64, _vp, _vp, _i64, _i64]),
    ("pcp_remove_duplicate", _i32, [_vp, _vp, _i64, _i32, _f32, _vp, _P(_i64)]),
    ("pcp_normals_knn", _i32, [_vp, _vp, _i32, _vp, _i64]),
    ("pcp_icp_create", _i32, [_vp, _vp, _vp, _sz, _i64, _P(_vp)]),
    ("pcp_icp_check_sizes", _i32, [_i64, _i64]),
    ("pcp_icp_destroy", _i32, [_vp]),
    ("pcp_icp_create_with_target", _i32, [_vp, _vp, _sz, _i64, _f64, _vp, _sz, _i64, _P(_vp), _P(_vp)]),
    ("pcp_icp_set_options", _i32, [_vp, _i32, _i32, _i32, _i32]),
    ("pcp_icp_step", _i32, [_vp, _vp, _P(_f64), _f32, _vp, _vp, _vp]),
    ("pcp_icp_keys", _i32, [_vp, _vp, _P(_f64), _f32, _i64, _vp]),
    ("pcp_icp_accumulate_keys", _i32, [_vp, _vp, _P(_f64), _vp, _i64, _i64, _vp, _sz, _vp]),
    ("pcp_icp_keys_dev", _i32, [_vp, _vp, _vp, _f32, _i64, _vp]),
    ("pcp_keys_owner", _i32, [_vp, _vp, _i64, _vp, _i32, _vp]),
    ("pcp_icp_accumulate_owned", _i32, [_vp, _vp, _vp, _sz, _i64, _vp, _vp, _i32, _i64, _i64, _vp, _sz, _vp]),
    ("pcp_slab_guard", _i32, [_vp, _vp, _P(_f64), _f64, _f64, _vp]),
    ("pcp_icp_solve", _i32, [_P(_f64), _i32, _P(_f64)]),
    ("pcp_icp_run", _i32, [_vp, _vp, _P(_f64), _f32, _i32, _i32, _f64, _P(_f32)]),
    ("pcp_icp_last_kernel_ms", _i32, [_vp, _P(_f64), _P(_i32)]),
    ("pcp_icp_step_dev", _i32, [_vp, _vp, _vp, _f32, _vp]),
    ("pcp_icp_solve_dev", _i32, [_vp, _vp, _i32, _vp, _vp]),
    ("pcp_icp_run_dev", _i32, [_vp, _vp, _vp, _f32, _i32, _i32, _vp]),
    ("pcp_icp_kernel_ms", _i32, [_vp, _vp, _P(_f64), _P(_i32)]),
    ("pcp_icp_last_fallback", _i32, [_vp, _P(_i64)]),
    ("pcp_icp_last_searched", _i32, [_vp, _P(_i64)]),
    ("pcp_fault_report_install", _i32, []),
    ("pcp_build_id", C.c_char_p, []),
    ("pcp_get_rot_icp", _i32, [_vp, _vp, _i64, _i32, _vp, _i64, _i32, _P(_f64), _f32, _i32, _i32,
                               _f64, _P(_f32)]),
]

_lib = None


class PcpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_STATUS.get(code, code)}: {msg}")
        self.code = code


def load(path=LIB_PATH, bind_all=True):
    """Load libpcp.so and bind every ABI symbol (raises if any is missing)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libpcp.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; "
            "g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = C.CDLL(path)
    if bind_all:
        skipped = []
        for name, res, args in SIGNATURES:
            if _AB and path == LIB_PATH and not hasattr(lib, name):  # an A/B build of an older tree
                skipped.append(name)
                continue
            fn = getattr(lib, name)  # AttributeError if the ABI symbol is missing
            fn.restype = res
            fn.argtypes = args
        if skipped:
            import sys
            print(f"_lib: A/B build {path} lacks {len(skipped)} ABI symbols: {', '.join(skipped)}", file=sys.stderr)
    if path == LIB_PATH:
        _lib = lib
    return lib


def check(rc, ctx=None):
    if rc != PCP_OK:
        msg = ""
        if ctx is not None:
            m = load().pcp_last_error(ctx)
            msg = m.decode() if m else ""
        raise PcpError(rc, msg)
    return rc


def f64arr(vals):
    vals = list(vals)
    return (C.c_double * len(vals))(*vals)
