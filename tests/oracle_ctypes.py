"""ctypes bindings to the CPU oracle (oracle/_build/libpcp_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "libpcp_oracle.so")

POINT48 = np.dtype(
    [("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("w", "<f8"), ("rgba", "<u4"),
     ("stamp_id", "<u4"), ("pad", "<u4", (2,))], align=False)
assert POINT48.itemsize == 48

PLANE = np.dtype([("normal_x", "<f4"), ("normal_y", "<f4"), ("normal_z", "<f4"),
                  ("min_value", "<f4"), ("curvature", "<f4"), ("distance", "<f4")])

_lib = None


def _ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def use_native():
    """bench.py cpu_baseline only: build the oracle on THIS host with -O3 -march=native
    (`make -C oracle native`, oracle/_build/native-<march>/) and make every later oracle call
    in this process use it.  Returns (path, march).  The parity build (-O2, portable) stays
    what tests/ and smoke() load."""
    global _lib
    out = subprocess.check_output(["make", "-s", "-C", ORACLE_DIR, "native"], text=True).strip().splitlines()
    path = os.path.join(ORACLE_DIR, out[-1])
    _lib = None
    load(path)
    return path, os.path.basename(os.path.dirname(path)).replace("native-", "")


def load(path=None):
    global _lib
    if _lib is not None and path is None:
        return _lib
    if path is None:
        path = LIB_PATH
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.ora_kdtree_build.restype = vp
    lib.ora_kdtree_build.argtypes = [vp, C.c_size_t, C.c_int, vp, C.c_int]
    lib.ora_kdtree_free.argtypes = [vp]
    lib.ora_kdtree_size.argtypes = [vp]
    lib.ora_kdtree_identity_mapping.argtypes = [vp]
    lib.ora_knn.argtypes = [vp, vp, C.c_int, vp, vp]
    lib.ora_knn_batch.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int, vp, vp, C.c_int]
    lib.ora_radius.argtypes = [vp, vp, C.c_double, C.c_uint, vp, vp, C.c_int]
    lib.ora_knn_lod.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp]
    lib.ora_getminmax3d.argtypes = [vp, C.c_int, C.c_int, vp, vp]
    lib.ora_centroid.argtypes = [vp, C.c_int, C.c_int, vp]
    lib.ora_centroid.restype = C.c_uint
    lib.ora_rpca.argtypes = [vp, C.c_size_t, C.c_int, vp, C.c_int, C.c_float, C.c_float, C.c_uint64, vp, C.c_int]
    lib.ora_rpca_draw.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
    lib.ora_rpca_draw.restype = C.c_uint32
    lib.ora_centroid_concat.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, vp]
    lib.ora_centroid_concat.restype = C.c_uint
    lib.ora_transform.argtypes = [vp, vp, C.c_int, C.c_int, vp]
    lib.ora_voxel_filter.argtypes = [vp, C.c_int, C.c_int, C.c_double, C.c_double,
                                     C.c_double, C.c_int, vp, vp]
    lib.ora_remove_duplicate.argtypes = [vp, C.c_int, C.c_int, C.c_float, vp]
    lib.ora_remove_duplicate_c.argtypes = [vp, C.c_int, C.c_int, C.c_float, vp, vp]
    lib.ora_plane_h_points.argtypes = [vp, C.c_int, vp]
    lib.ora_normals_knn.argtypes = [vp, vp, C.c_size_t, C.c_int, C.c_int, vp, C.c_int]
    lib.ora_radius_normals_batch.argtypes = [vp, vp, C.c_size_t, vp, C.c_int, C.c_double, vp, vp, C.c_int]
    lib.ora_eigen_sym3.argtypes = [vp, vp, vp]
    lib.ora_f32index_build.restype = vp
    lib.ora_f32index_build.argtypes = [vp, C.c_int]
    lib.ora_f32index_free.argtypes = [vp]
    lib.ora_icp_correspond.argtypes = [vp, vp, C.c_int, vp, vp, C.c_float, vp, vp, C.c_int]
    lib.ora_icp_accumulate.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp]
    lib.ora_icp_solve.argtypes = [vp, C.c_int, vp]
    lib.ora_icp.restype = C.c_double
    lib.ora_icp.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_float, C.c_int, C.c_int, C.c_int]
    lib.ora_icp_timed.restype = C.c_double
    lib.ora_icp_timed.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_float, C.c_int, C.c_int, C.c_int,
                                  C.c_int, vp, vp]
    lib.ora_get_rot_icp.restype = C.c_float
    lib.ora_get_rot_icp.argtypes = [vp, C.c_int, C.c_int, vp, C.c_int, C.c_int, vp, C.c_float,
                                    C.c_int, C.c_int, C.c_int]
    lib.ora_grid_create.restype = vp
    lib.ora_grid_free.argtypes = [vp]
    lib.ora_grid_add_cloud.argtypes = [vp, vp, C.c_int]
    lib.ora_grid_size.argtypes = [vp]
    lib.ora_grid_points.argtypes = [vp, vp]
    lib.ora_grid_box.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    lib.ora_grid_match.argtypes = [vp, vp, C.c_int, C.c_float, vp, vp, vp]
    _lib = lib
    return lib


def make_cloud(xyz, rgba=None, stamp=None):
    """AoS48 PointXYZRGBA array from an (n,3) array."""
    xyz = np.asarray(xyz, dtype=np.float64).reshape(-1, 3)
    c = np.zeros(len(xyz), dtype=POINT48)
    c["x"], c["y"], c["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    c["w"] = 1.0
    if rgba is not None:
        c["rgba"] = rgba
    if stamp is not None:
        c["stamp_id"] = stamp
    return c


class KdTree:
    """Oracle KdTreeFLANN (double)."""

    def __init__(self, xyz, stride=3, n=None, indices=None):
        self.lib = load()
        self.xyz = np.ascontiguousarray(xyz, dtype=np.float64)
        n = len(self.xyz) if n is None else n
        self.indices = None if indices is None else np.ascontiguousarray(indices, dtype=np.int32)
        self.h = self.lib.ora_kdtree_build(
            self.xyz.ctypes.data, stride, n,
            None if self.indices is None else self.indices.ctypes.data,
            0 if self.indices is None else len(self.indices))

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ora_kdtree_free(self.h)
            self.h = None

    @property
    def size(self):
        return self.lib.ora_kdtree_size(self.h)

    def knn(self, q, k, nthreads=0):
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, 3)
        idx = np.empty((len(q), k), np.int32)
        d2 = np.empty((len(q), k), np.float64)
        self.lib.ora_knn_batch(self.h, q.ctypes.data, 3, len(q), k, idx.ctypes.data,
                               d2.ctypes.data, int(nthreads))
        return idx, d2

    def radius_normals(self, qidx, r, nthreads=0):
        """C5 CPU leg: radiusSearch(r) of the tree's own points qidx + F1 per row (OpenMP).
        The tree must be built over its (n, 3) xyz with stride 3."""
        qidx = np.ascontiguousarray(qidx, dtype=np.int32)
        cnt = np.empty(max(len(qidx), 1), np.int32)
        planes = np.empty(max(len(qidx), 1), PLANE)
        self.lib.ora_radius_normals_batch(self.h, self.xyz.ctypes.data, 3, qidx.ctypes.data, len(qidx), float(r),
                                          cnt.ctypes.data, planes.ctypes.data, int(nthreads))
        return cnt[:len(qidx)], planes[:len(qidx)]

    def radius(self, q, r, max_nn=0, cap=None):
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(3)
        cap = self.size if cap is None else cap
        idx = np.empty(max(cap, 1), np.int32)
        d2 = np.empty(max(cap, 1), np.float64)
        cnt = self.lib.ora_radius(self.h, q.ctypes.data, float(r), int(max_nn),
                                  idx.ctypes.data, d2.ctypes.data, cap)
        return idx[:cnt], d2[:cnt]


def voxel_filter(cloud, leaf, is_dense=True, downsample_all=True):
    lib = load()
    cloud = np.ascontiguousarray(cloud)
    out = np.zeros(max(len(cloud), 1), dtype=POINT48)
    vidx = np.zeros(max(len(cloud), 1), dtype=np.uint32)
    lx, ly, lz = (leaf, leaf, leaf) if np.isscalar(leaf) else leaf
    m = lib.ora_voxel_filter(cloud.ctypes.data, len(cloud), int(is_dense), lx, ly, lz,
                             int(downsample_all), out.ctypes.data, vidx.ctypes.data)
    return out[:m], vidx[:m]


def remove_duplicate(cloud, leaf, is_dense=True):
    lib = load()
    cloud = np.ascontiguousarray(cloud)
    out = np.zeros(max(len(cloud), 1), dtype=POINT48)
    m = lib.ora_remove_duplicate(cloud.ctypes.data, len(cloud), int(is_dense),
                                 float(leaf), out.ctypes.data)
    return out[:m]


def remove_duplicate_c(cloud, leaf, c, is_dense=True):
    lib = load()
    cloud = np.ascontiguousarray(cloud)
    out = np.zeros(max(len(cloud), 1), dtype=POINT48)
    c = np.ascontiguousarray(np.asarray(c, dtype=np.float64)[:3])
    m = lib.ora_remove_duplicate_c(cloud.ctypes.data, len(cloud), int(is_dense), float(leaf),
                                   c.ctypes.data, out.ctypes.data)
    return out[:m]


def centroid(cloud, is_dense=True):
    lib = load()
    c = np.zeros(4)
    lib.ora_centroid(np.ascontiguousarray(cloud).ctypes.data, len(cloud), int(is_dense),
                     c.ctypes.data)
    return c


def centroid_concat(a, b, is_dense=True):
    lib = load()
    c = np.zeros(4)
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    lib.ora_centroid_concat(a.ctypes.data, len(a), b.ctypes.data, len(b), int(is_dense), c.ctypes.data)
    return c


POINT_PROPERTY = np.dtype([("normal_x", "<f4"), ("normal_y", "<f4"), ("normal_z", "<f4"), ("pad", "<u4"),
                           ("distance", "<f8"), ("curvature", "<f8"), ("point_id", "<i4"),
                           ("segment_id", "<i4"), ("dis_from_point_plane", "<f4"), ("pad2", "<u4")])


def rpca(xyz, knn_idx, pr=0.99, epi=0.5, seed=0, nthreads=0):
    """F3 calculate_plan_parameter_rpca restated (ora_rpca) from kNN rows (n, k)."""
    lib = load()
    xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
    knn_idx = np.ascontiguousarray(knn_idx, dtype=np.int32)
    out = np.zeros(len(xyz), dtype=POINT_PROPERTY)
    lib.ora_rpca(xyz.ctypes.data, 3, len(xyz), knn_idx.ctypes.data, knn_idx.shape[1], float(pr), float(epi),
                 int(seed), out.ctypes.data, nthreads)
    return out


def minmax(cloud, is_dense=True):
    lib = load()
    mn, mx = np.zeros(4), np.zeros(4)
    lib.ora_getminmax3d(np.ascontiguousarray(cloud).ctypes.data, len(cloud), int(is_dense),
                        mn.ctypes.data, mx.ctypes.data)
    return mn, mx


def transform(cloud, T, is_dense=True):
    lib = load()
    cloud = np.ascontiguousarray(cloud)
    out = np.zeros_like(cloud)
    T = np.ascontiguousarray(T, dtype=np.float64)
    lib.ora_transform(cloud.ctypes.data, out.ctypes.data, len(cloud), int(is_dense),
                      T.ctypes.data)
    return out


def normals_knn(xyz, k, nthreads=0):
    lib = load()
    xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
    t = KdTree(xyz)
    out = np.zeros(len(xyz), dtype=PLANE)
    lib.ora_normals_knn(t.h, xyz.ctypes.data, 3, len(xyz), k, out.ctypes.data, nthreads)
    return out


def knn_lod(cloud, q, k):
    lib = load()
    cloud = np.ascontiguousarray(cloud)
    qa = np.ascontiguousarray(np.asarray(q).reshape(1)) if getattr(q, "dtype", None) == POINT48 \
        else make_cloud(np.asarray(q).reshape(1, 3))
    idx = np.empty(max(k, 1), np.int32)
    d2 = np.empty(max(k, 1), np.float64)
    n = lib.ora_knn_lod(cloud.ctypes.data, len(cloud), qa.ctypes.data, k, idx.ctypes.data,
                        d2.ctypes.data)
    return idx[:n], d2[:n]


class F32Index:
    def __init__(self, xyz):
        self.lib = load()
        self.xyz = np.ascontiguousarray(xyz, dtype=np.float32).reshape(-1, 3)
        self.h = self.lib.ora_f32index_build(self.xyz.ctypes.data, len(self.xyz))

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ora_f32index_free(self.h)
            self.h = None

    def correspond(self, q, R, t, rmax, nthreads=0):
        q = np.ascontiguousarray(q, dtype=np.float32).reshape(-1, 3)
        R = np.ascontiguousarray(R, dtype=np.float32).reshape(9)
        t = np.ascontiguousarray(t, dtype=np.float32).reshape(3)
        idx = np.empty(len(q), np.int32)
        d2 = np.empty(len(q), np.float32)
        self.lib.ora_icp_correspond(self.h, q.ctypes.data, len(q), R.ctypes.data, t.ctypes.data,
                                    float(rmax), idx.ctypes.data, d2.ctypes.data, nthreads)
        return idx, d2


def icp_accumulate(tgt, q, R, t, idx, d2):
    lib = load()
    tgt = np.ascontiguousarray(tgt, dtype=np.float32)
    q = np.ascontiguousarray(q, dtype=np.float32)
    R = np.ascontiguousarray(R, dtype=np.float32).reshape(9)
    t = np.ascontiguousarray(t, dtype=np.float32).reshape(3)
    acc = np.zeros(24)
    lib.ora_icp_accumulate(tgt.ctypes.data, q.ctypes.data, len(q), R.ctypes.data, t.ctypes.data,
                           np.ascontiguousarray(idx, np.int32).ctypes.data,
                           np.ascontiguousarray(d2, np.float32).ctypes.data, acc.ctypes.data)
    return acc


def icp_solve(acc, do_scale=False):
    lib = load()
    acc = np.ascontiguousarray(acc, dtype=np.float64)
    dT = np.zeros(16)
    rc = lib.ora_icp_solve(acc.ctypes.data, int(do_scale), dT.ctypes.data)
    return rc, dT.reshape(4, 4)


def icp_timed(tgt, q, T0, rmax, iters, do_scale=False, nthreads=0):
    """CPU-baseline ICP: returns (err, T, build_s, iter_s) with per-thread accumulators."""
    lib = load()
    tgt = np.ascontiguousarray(tgt, dtype=np.float32).reshape(-1, 3)
    q = np.ascontiguousarray(q, dtype=np.float32).reshape(-1, 3)
    T = np.ascontiguousarray(np.array(T0, dtype=np.float64).reshape(16))
    bs, its = C.c_double(), C.c_double()
    err = lib.ora_icp_timed(tgt.ctypes.data, len(tgt), q.ctypes.data, len(q), T.ctypes.data, float(rmax),
                            int(iters), int(do_scale), int(nthreads), 1, C.byref(bs), C.byref(its))
    return err, T.reshape(4, 4), bs.value, its.value


def icp(tgt, q, T0, rmax, iters, do_scale=False, nthreads=0):
    lib = load()
    tgt = np.ascontiguousarray(tgt, dtype=np.float32).reshape(-1, 3)
    q = np.ascontiguousarray(q, dtype=np.float32).reshape(-1, 3)
    T = np.ascontiguousarray(np.array(T0, dtype=np.float64).reshape(16))
    err = lib.ora_icp(tgt.ctypes.data, len(tgt), q.ctypes.data, len(q), T.ctypes.data,
                      float(rmax), int(iters), int(do_scale), nthreads)
    return err, T.reshape(4, 4)


def get_rot_icp(src, tmp, rmax, iters, do_scale=False, nthreads=0, src_dense=True, tmp_dense=True):
    lib = load()
    src = np.ascontiguousarray(src)
    tmp = np.ascontiguousarray(tmp)
    M = np.zeros(16)
    err = lib.ora_get_rot_icp(src.ctypes.data, len(src), int(src_dense), tmp.ctypes.data, len(tmp),
                              int(tmp_dense), M.ctypes.data, float(rmax), int(iters), int(do_scale),
                              nthreads)
    return float(err), M.reshape(4, 4)


class Grid:
    """CloudGrid restatement (ora_grid_*, cloud_grid.cpp)."""

    def __init__(self):
        self.lib = load()
        self.h = self.lib.ora_grid_create()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ora_grid_free(self.h)
            self.h = None

    def add_cloud(self, cloud):
        cloud = np.ascontiguousarray(cloud)
        self.lib.ora_grid_add_cloud(self.h, cloud.ctypes.data, len(cloud))

    @property
    def size(self):
        return self.lib.ora_grid_size(self.h)

    def points(self):
        out = np.zeros(max(self.size, 1), dtype=POINT48)
        m = self.lib.ora_grid_points(self.h, out.ctypes.data)
        return out[:m]

    def box(self, i0, i1, j0, j1):
        out = np.zeros(max(self.size, 1), dtype=POINT48)
        m = self.lib.ora_grid_box(self.h, int(i0), int(i1), int(j0), int(j1), out.ctypes.data)
        return out[:m]

    def match(self, src, dis):
        src = np.ascontiguousarray(src)
        so = np.zeros(max(len(src), 1), dtype=POINT48)
        dst = np.zeros(max(self.size, 1), dtype=POINT48)
        ns = C.c_int(0)
        nd = self.lib.ora_grid_match(self.h, src.ctypes.data, len(src), C.c_float(dis), so.ctypes.data,
                                     C.byref(ns), dst.ctypes.data)
        return so[:ns.value], dst[:nd]
