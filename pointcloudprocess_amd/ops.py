"""Python host layer over the C-ABI (include/pcp.h) for device-resident clouds.

torch is plumbing only: it owns device memory and the stream; every computation is a
libpcp HIP kernel.  Clouds in the reference layout (PointXYZRGBA, point_type.h:9-82) are
uint8 tensors of shape (n, 48); xyz clouds are float64/float32 tensors of shape (n, 3).
"""
import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import check

POINT48 = np.dtype(
    [("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("w", "<f8"), ("rgba", "<u4"),
     ("stamp_id", "<u4"), ("pad", "<u4", (2,))])
PLANE = np.dtype([("normal_x", "<f4"), ("normal_y", "<f4"), ("normal_z", "<f4"),
                  ("min_value", "<f4"), ("curvature", "<f4"), ("distance", "<f4")])


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class Context:
    """pcp_ctx bound to a device and to torch's current stream on that device."""

    def __init__(self, device=0):
        self.lib = _lib.load()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        idx = self.device.index or 0
        stream = torch.cuda.current_stream(self.device).cuda_stream
        h = C.c_void_p()
        rc = self.lib.pcp_ctx_create(idx, C.c_void_p(stream), C.byref(h))
        if rc != 0:
            raise _lib.PcpError(rc, f"pcp_ctx_create(device={idx}) failed")
        self.h = h

    def check(self, rc):
        return check(rc, self.h)

    def sync(self):
        self.check(self.lib.pcp_sync(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.lib.pcp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def cloud_to_device(cloud_np, device):
    """numpy POINT48 structured array -> (n, 48) uint8 device tensor."""
    arr = np.ascontiguousarray(cloud_np)
    assert arr.dtype.itemsize == 48
    t = torch.from_numpy(arr.view(np.uint8).reshape(len(arr), 48))
    return t.to(device)


def cloud_to_host(t):
    a = t.detach().cpu().contiguous().numpy().reshape(-1)
    return a.view(POINT48)


class GridIndex:
    """pcp_index over a cloud.  fp64 (KdTreeFLANN contract) or fp32 (ICP target)."""

    def __init__(self, ctx, xyz, cell_size=0.0, indices=None, stride_bytes=None):
        self.ctx = ctx
        lib = ctx.lib
        self.src = xyz  # keep alive
        h = C.c_void_p()
        n = xyz.shape[0]
        if xyz.dtype == torch.uint8:  # AoS48
            stride = 48
            self.f64 = True
        else:
            self.f64 = xyz.dtype == torch.float64
            stride = stride_bytes or xyz.stride(0) * xyz.element_size()
        if self.f64:
            self.indices = None if indices is None else indices.to(ctx.device, torch.int32).contiguous()
            ni = 0 if self.indices is None else self.indices.numel()
            ctx.check(lib.pcp_index_build_f64(ctx.h, _ptr(xyz), stride, n, _ptr(self.indices), ni,
                                              float(cell_size), C.byref(h)))
        else:
            if indices is not None:
                raise ValueError("fp32 index does not take an indices subset")
            ctx.check(lib.pcp_index_build_f32(ctx.h, _ptr(xyz), stride, n, float(cell_size), C.byref(h)))
        self.h = h

    @property
    def size(self):
        return self.ctx.lib.pcp_index_size(self.h)

    @property
    def cell_size(self):
        return self.ctx.lib.pcp_index_cell_size(self.h)

    @property
    def identity_mapping(self):
        return bool(self.ctx.lib.pcp_index_identity_mapping(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.pcp_index_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def _qstride(q):
    if q.dtype == torch.uint8:
        return 48
    return q.stride(0) * q.element_size()


def knn(index, q, k):
    """Batch nearestKSearch: (nq, k) int32 indices and float64 sqr distances."""
    ctx = index.ctx
    nq = q.shape[0]
    idx = torch.empty((nq, k), dtype=torch.int32, device=ctx.device)
    d2 = torch.empty((nq, k), dtype=torch.float64, device=ctx.device)
    ctx.check(ctx.lib.pcp_knn(ctx.h, index.h, _ptr(q), _qstride(q), nq, int(k), _ptr(idx), _ptr(d2)))
    return idx, d2


def radius(index, q, r, max_nn=0):
    """Batch radiusSearch -> CSR (offsets int64 (nq+1), idx int32, d2 float64)."""
    ctx = index.ctx
    nq = q.shape[0]
    cnt = torch.empty(nq, dtype=torch.int32, device=ctx.device)
    ctx.check(ctx.lib.pcp_radius_count(ctx.h, index.h, _ptr(q), _qstride(q), nq, float(r), int(max_nn),
                                       _ptr(cnt)))
    offs = torch.empty(nq + 1, dtype=torch.int64, device=ctx.device)
    total = C.c_int64()
    ctx.check(ctx.lib.pcp_scan_counts(ctx.h, _ptr(cnt), nq, _ptr(offs), C.byref(total)))
    idx = torch.empty(max(total.value, 1), dtype=torch.int32, device=ctx.device)
    d2 = torch.empty(max(total.value, 1), dtype=torch.float64, device=ctx.device)
    ctx.check(ctx.lib.pcp_radius_fill(ctx.h, index.h, _ptr(q), _qstride(q), nq, float(r), int(max_nn),
                                      _ptr(offs), _ptr(idx), _ptr(d2)))
    return offs, idx[:total.value], d2[:total.value]


class H16Index:
    """C5 fp16 cell-relative index over an (n, 3) fp32 cloud (pcp_index_build_h16)."""

    def __init__(self, ctx, xyz, cell_size):
        self.ctx = ctx
        self.src = xyz
        h = C.c_void_p()
        ctx.check(ctx.lib.pcp_index_build_h16(ctx.h, _ptr(xyz), xyz.stride(0) * xyz.element_size(), xyz.shape[0],
                                              float(cell_size), C.byref(h)))
        self.h = h

    def radius_normals(self, r, n_owned=None, global_id=None, normals=True):
        """Rows (offsets int64 (n_owned+1), idx int32) of the owned points + their planes."""
        ctx = self.ctx
        n_owned = self.src.shape[0] if n_owned is None else int(n_owned)
        cnt = torch.empty(max(n_owned, 1), dtype=torch.int32, device=ctx.device)
        ctx.check(ctx.lib.pcp_h16_radius_count(ctx.h, self.h, float(r), n_owned, _ptr(cnt)))
        offs = torch.empty(n_owned + 1, dtype=torch.int64, device=ctx.device)
        total = C.c_int64()
        ctx.check(ctx.lib.pcp_scan_counts(ctx.h, _ptr(cnt), n_owned, _ptr(offs), C.byref(total)))
        idx = torch.empty(max(total.value, 1), dtype=torch.int32, device=ctx.device)
        nrm = torch.empty((max(n_owned, 1), 6), dtype=torch.float32, device=ctx.device) if normals else None
        ctx.check(ctx.lib.pcp_h16_radius_fill(ctx.h, self.h, float(r), n_owned, _ptr(offs), _ptr(global_id),
                                              _ptr(idx), _ptr(nrm)))
        return offs, idx[:total.value], (nrm[:n_owned] if normals else None)

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.pcp_index_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def nearest_query(index, q, init_bound=9999.0):
    """find_cloud_nearest_point_in_kdtree: (query index or -1, its 1-NN d2)."""
    ctx = index.ctx
    bq, bd = C.c_int64(), C.c_double()
    ctx.check(ctx.lib.pcp_nearest_query(ctx.h, index.h, _ptr(q), _qstride(q), q.shape[0], float(init_bound),
                                        C.byref(bq), C.byref(bd)))
    return bq.value, bd.value


def plane_fit_segments(ctx, xyz, offsets, idx=None):
    """One PlanSegment per CSR segment of xyz rows (F1 per segment)."""
    nseg = offsets.numel() - 1
    out = torch.empty((max(nseg, 1), 6), dtype=torch.float32, device=ctx.device)
    ctx.check(ctx.lib.pcp_plane_fit_segments(ctx.h, _ptr(xyz), _qstride(xyz), _ptr(offsets), _ptr(idx), nseg,
                                             _ptr(out)))
    return out[:nseg]


def normals_radius(index, r, max_nn=0):
    """calculate_plan_parameter(cloud, radius) (calculate_feature.h:15, declared-only in the
    reference; the build defines it as F1 over each point's radiusSearch neighbourhood)."""
    xyz = index.src
    offs, idx, _ = radius(index, xyz, r, max_nn)
    return plane_fit_segments(index.ctx, xyz, offs, idx)


def knn_bruteforce(ctx, target, q, k):
    nt, nq = target.shape[0], q.shape[0]
    idx = torch.empty((nq, k), dtype=torch.int32, device=ctx.device)
    d2 = torch.empty((nq, k), dtype=torch.float64, device=ctx.device)
    ctx.check(ctx.lib.pcp_knn_bruteforce(ctx.h, _ptr(target), _qstride(target), nt, _ptr(q), _qstride(q),
                                         nq, int(k), _ptr(idx), _ptr(d2)))
    return idx, d2


def knn_bruteforce_last_fallback(ctx):
    n = C.c_int64()
    ctx.check(ctx.lib.pcp_knn_bruteforce_last_fallback(ctx.h, C.byref(n)))
    return n.value


def knn_lod(ctx, cloud, q, k):
    nq = q.shape[0]
    idx = torch.empty((nq, k), dtype=torch.int32, device=ctx.device)
    d2 = torch.empty((nq, k), dtype=torch.float64, device=ctx.device)
    ctx.check(ctx.lib.pcp_knn_lod(ctx.h, _ptr(cloud), cloud.shape[0], _ptr(q), nq, int(k), _ptr(idx),
                                  _ptr(d2)))
    return idx, d2


def minmax(ctx, cloud, is_dense=True):
    mn, mx = (C.c_double * 4)(), (C.c_double * 4)()
    ctx.check(ctx.lib.pcp_minmax_aos48(ctx.h, _ptr(cloud), cloud.shape[0], int(is_dense), mn, mx))
    return np.array(mn[:]), np.array(mx[:])


def centroid(ctx, cloud, is_dense=True):
    c = (C.c_double * 4)()
    cnt = C.c_uint32()
    ctx.check(ctx.lib.pcp_centroid_aos48(ctx.h, _ptr(cloud), cloud.shape[0], int(is_dense), c,
                                         C.byref(cnt)))
    return np.array(c[:]), cnt.value


def centroid_concat(ctx, a, b, is_dense=True):
    """compute3DCentroid of a ++ b (the joint centroid of get_rot_icp)."""
    c = (C.c_double * 4)()
    cnt = C.c_uint32()
    ctx.check(ctx.lib.pcp_centroid_concat_aos48(ctx.h, _ptr(a), a.shape[0], _ptr(b), b.shape[0], int(is_dense),
                                                c, C.byref(cnt)))
    return np.array(c[:]), cnt.value


def transform(ctx, cloud, T, is_dense=True, out=None):
    out = torch.empty_like(cloud) if out is None else out
    Tm = _lib.f64arr(np.asarray(T, dtype=np.float64).reshape(16))
    ctx.check(ctx.lib.pcp_transform_aos48(ctx.h, _ptr(cloud), _ptr(out), cloud.shape[0], int(is_dense), Tm))
    return out


def voxel_filter(ctx, cloud, leaf, is_dense=True, downsample_all=True, with_voxel_idx=False):
    n = cloud.shape[0]
    out = torch.empty((max(n, 1), 48), dtype=torch.uint8, device=ctx.device)
    vidx = torch.empty(max(n, 1), dtype=torch.int32, device=ctx.device) if with_voxel_idx else None
    lf = (leaf, leaf, leaf) if np.isscalar(leaf) else tuple(leaf)
    nout = C.c_int64()
    ctx.check(ctx.lib.pcp_voxel_filter(ctx.h, _ptr(cloud), n, int(is_dense), _lib.f64arr(lf),
                                       int(downsample_all), _ptr(out), C.byref(nout), _ptr(vidx)))
    m = nout.value
    if with_voxel_idx:
        return out[:m], vidx[:m].view(torch.int32)
    return out[:m]


def remove_duplicate(ctx, cloud, leaf, is_dense=True):
    n = cloud.shape[0]
    out = torch.empty((max(n, 1), 48), dtype=torch.uint8, device=ctx.device)
    nout = C.c_int64()
    ctx.check(ctx.lib.pcp_remove_duplicate(ctx.h, _ptr(cloud), n, int(is_dense), float(leaf), _ptr(out),
                                           C.byref(nout)))
    return out[:nout.value]


def normals_knn(index, k):
    ctx = index.ctx
    n_out = index.src.shape[0]  # outputs are indexed by the caller's cloud index
    out = torch.empty((max(n_out, 1), 6), dtype=torch.float32, device=ctx.device)
    ctx.check(ctx.lib.pcp_normals_knn(ctx.h, index.h, int(k), _ptr(out), n_out))
    return out[:n_out]


POINT_PROPERTY = np.dtype([("normal_x", "<f4"), ("normal_y", "<f4"), ("normal_z", "<f4"), ("pad", "<u4"),
                           ("distance", "<f8"), ("curvature", "<f8"), ("point_id", "<i4"),
                           ("segment_id", "<i4"), ("dis_from_point_plane", "<f4"), ("pad2", "<u4")])


def normals_rpca(ctx, xyz, knn_idx, pr=0.99, epi=0.5, seed=0):
    """F3 robust normals (calculate_plan_parameter_rpca) from the cloud's kNN(20) rows;
    returns a (n, 48) uint8 device tensor of LAS_POINT_PROPERTY records."""
    n = xyz.shape[0]
    k = knn_idx.shape[1]
    out = torch.empty((max(n, 1), 48), dtype=torch.uint8, device=ctx.device)
    ctx.check(ctx.lib.pcp_normals_rpca(ctx.h, _ptr(xyz), xyz.stride(0) * xyz.element_size(), n,
                                       _ptr(knn_idx.contiguous()), int(k), float(pr), float(epi),
                                       int(seed), _ptr(out)))
    return out[:n]


class ICP:
    """Device-resident ICP of a query set against an fp32 grid index (the target)."""

    def __init__(self, target_index, q, _handle=None):
        self.index = target_index
        self.ctx = ctx = target_index.ctx
        self.q = q
        h = C.c_void_p()
        if _handle is None:
            ctx.check(ctx.lib.pcp_icp_create(ctx.h, target_index.h, _ptr(q), q.stride(0) * q.element_size(),
                                             q.shape[0], C.byref(h)))
        else:
            h = _handle
        self.h = h
        self.nq_in = q.shape[0]
        self.acc = torch.zeros(24, dtype=torch.float64, device=ctx.device)

    @classmethod
    def with_target(cls, ctx, target, q, cell_size):
        """The fp32 index of `target` and the ICP handle of `q` in one call
        (pcp_icp_create_with_target: the two pre-iteration sorts overlap).  Returns the ICP; its
        .index is the GridIndex (close the ICP, then the index)."""
        hi, hq = C.c_void_p(), C.c_void_p()
        ctx.check(ctx.lib.pcp_icp_create_with_target(ctx.h, _ptr(target), target.stride(0) * target.element_size(),
                                                     target.shape[0], float(cell_size), _ptr(q),
                                                     q.stride(0) * q.element_size(), q.shape[0], C.byref(hi),
                                                     C.byref(hq)))
        index = GridIndex.__new__(GridIndex)
        index.ctx, index.src, index.h, index.f64, index.indices = ctx, target, hi, False, None
        return cls(index, q, _handle=hq)

    WIDE_CACHE = 128  # PCP_ICP_OPT_WIDE_CACHE
    GRAPH = 256       # PCP_ICP_OPT_GRAPH

    def set_options(self, oct_lanes_first=1, oct_lanes_list=0, ring_lanes=0, ablate=0, wide_cache=False,
                    graph=False):
        """Test / profiling controls (pcp_icp_set_options): lanes per query of the octant pass
        (first launch, later lists; 0 = by density) and of the fallback pass (0 = by length);
        `ablate` switches passes off (results are then wrong); `wide_cache` keeps 16-byte cache
        records (before the first step); `graph` replays one captured HIP graph per device-pose
        launch (results are identical in both cases)."""
        flags = int(ablate) | (self.WIDE_CACHE if wide_cache else 0) | (self.GRAPH if graph else 0)
        self.ctx.check(self.ctx.lib.pcp_icp_set_options(self.h, int(oct_lanes_first), int(oct_lanes_list),
                                                        int(ring_lanes), flags))

    def step(self, T, rmax, corr=False):
        """One iteration at pose T; returns the (device) accumulators (+ correspondences)."""
        ctx = self.ctx
        Tm = _lib.f64arr(np.asarray(T, dtype=np.float64).reshape(16))
        ci = cd = None
        if corr:
            ci = torch.empty(self.q.shape[0], dtype=torch.int32, device=ctx.device)
            cd = torch.empty(self.q.shape[0], dtype=torch.float32, device=ctx.device)
        ctx.check(ctx.lib.pcp_icp_step(ctx.h, self.h, Tm, float(rmax), _ptr(self.acc), _ptr(ci), _ptr(cd)))
        return (self.acc, ci, cd) if corr else self.acc

    def run(self, T0, rmax, iters, do_scale=False, eps=0.0):
        ctx = self.ctx
        T = _lib.f64arr(np.asarray(T0, dtype=np.float64).reshape(16))
        err = C.c_float()
        rc = ctx.lib.pcp_icp_run(ctx.h, self.h, T, float(rmax), int(iters), int(do_scale), float(eps),
                                 C.byref(err))
        if rc not in (0, -6):
            ctx.check(rc)
        return float(err.value), np.array(T[:]).reshape(4, 4)

    # ---- device-resident loop: the pose stays in HBM, no host round trip per iteration
    def new_pose(self, T0=None):
        """(T_dev, stats_dev): a device pose (16 fp64, row-major) and zeroed stats (4 fp64)."""
        T = torch.as_tensor(np.eye(4) if T0 is None else np.asarray(T0, dtype=np.float64), dtype=torch.float64)
        return T.reshape(16).to(self.ctx.device).contiguous(), torch.zeros(4, dtype=torch.float64,
                                                                        device=self.ctx.device)

    def step_dev(self, T_dev, rmax):
        ctx = self.ctx
        ctx.check(ctx.lib.pcp_icp_step_dev(ctx.h, self.h, _ptr(T_dev), float(rmax), _ptr(self.acc)))
        return self.acc

    def solve_dev(self, acc, T_dev, stats, do_scale=False):
        ctx = self.ctx
        ctx.check(ctx.lib.pcp_icp_solve_dev(ctx.h, _ptr(acc), int(do_scale), _ptr(T_dev), _ptr(stats)))

    def run_dev(self, T_dev, stats, rmax, iters, do_scale=False):
        ctx = self.ctx
        ctx.check(ctx.lib.pcp_icp_run_dev(ctx.h, self.h, _ptr(T_dev), float(rmax), int(iters), int(do_scale),
                                          _ptr(stats)))

    def kernel_ms(self):
        """(ms, launches) of the device-loop correspondence kernels since the last call."""
        ms, n = C.c_double(), C.c_int()
        self.ctx.check(self.ctx.lib.pcp_icp_kernel_ms(self.ctx.h, self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def keys(self, T, rmax, target_offset=0):
        """Target-sharded mode: per-query int64 keys (fp32 d2 bits << 32 | global target
        index, INT64_MAX = none) in the original query order."""
        ctx = self.ctx
        keys = torch.empty(self.nq_in, dtype=torch.int64, device=ctx.device)
        Tm = _lib.f64arr(np.asarray(T, dtype=np.float64).reshape(16))
        ctx.check(ctx.lib.pcp_icp_keys(ctx.h, self.h, Tm, float(rmax), int(target_offset), _ptr(keys)))
        return keys

    def keys_dev(self, T_dev, rmax, target_offset=0, out=None):
        """keys() at the device pose T_dev (no host round trip)."""
        ctx = self.ctx
        keys = torch.empty(self.nq_in, dtype=torch.int64, device=ctx.device) if out is None else out
        assert keys.dtype == torch.int64 and keys.numel() >= self.nq_in and keys.is_contiguous()
        ctx.check(ctx.lib.pcp_icp_keys_dev(ctx.h, self.h, _ptr(T_dev), float(rmax), int(target_offset), _ptr(keys)))
        return keys

    def accumulate_keys(self, T, keys, lo, hi, shard_xyz):
        """24 accumulators of the queries whose (MIN-reduced) winner is in [lo, hi)."""
        ctx = self.ctx
        Tm = _lib.f64arr(np.asarray(T, dtype=np.float64).reshape(16))
        ctx.check(ctx.lib.pcp_icp_accumulate_keys(ctx.h, self.h, Tm, _ptr(keys), int(lo), int(hi), _ptr(shard_xyz),
                                                  shard_xyz.stride(0) * shard_xyz.element_size(), _ptr(self.acc)))
        return self.acc

    def last_kernel_ms(self):
        ms, n = C.c_double(), C.c_int()
        self.ctx.check(self.ctx.lib.pcp_icp_last_kernel_ms(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def last_searched(self):
        """Queries of the last step the verify pass could not settle (they were searched)."""
        n = C.c_int64()
        self.ctx.check(self.ctx.lib.pcp_icp_last_searched(self.h, C.byref(n)))
        return n.value

    def last_fallback(self):
        n = C.c_int64()
        self.ctx.check(self.ctx.lib.pcp_icp_last_fallback(self.h, C.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.pcp_icp_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def keys_owner(ctx, keys, bounds, out=None):
    """Per key (int64, global target index in the low 32 bits), the shard owning its winner:
    s with bounds[s] <= index < bounds[s + 1] (bounds: int64 device tensor, nshards + 1), 255
    for no correspondence.  uint8 device tensor."""
    n = keys.numel()
    out = torch.empty(n, dtype=torch.uint8, device=ctx.device) if out is None else out
    assert keys.dtype == torch.int64 and bounds.dtype == torch.int64 and out.numel() >= n
    ctx.check(ctx.lib.pcp_keys_owner(ctx.h, _ptr(keys), n, _ptr(bounds), bounds.numel() - 1, _ptr(out)))
    return out


def accumulate_owned(ctx, T_dev, q, keys, owner, rank, lo, hi, shard_xyz, acc=None):
    """Accumulators of the queries q (n x 3 fp32, ALL queries, original order) whose winner
    this rank owns (owner == rank), read from its own shard (global indices [lo, hi)) through
    its local keys: the device-resident target-sharded loop's accumulation."""
    acc = torch.zeros(24, dtype=torch.float64, device=ctx.device) if acc is None else acc
    n = q.shape[0]
    assert keys.numel() >= n and keys.dtype == torch.int64 and owner.numel() >= n and owner.dtype == torch.uint8
    ctx.check(ctx.lib.pcp_icp_accumulate_owned(ctx.h, _ptr(T_dev), _ptr(q) if n else None,
                                               q.stride(0) * q.element_size(), n, _ptr(keys), _ptr(owner), int(rank),
                                               int(lo), int(hi), _ptr(shard_xyz),
                                               shard_xyz.stride(0) * shard_xyz.element_size(), _ptr(acc)))
    return acc


def slab_guard(ctx, T_dev, box, lo, hi, flag):
    """Latch flag[0] = 1 when the owned queries' box leaves x in [lo, hi] under T_dev."""
    ctx.check(ctx.lib.pcp_slab_guard(ctx.h, _ptr(T_dev), _lib.f64arr(np.asarray(box, dtype=np.float64).reshape(6)),
                                     float(lo), float(hi), _ptr(flag)))


def icp_solve(acc, do_scale=False):
    a = np.asarray(acc, dtype=np.float64).reshape(24)
    dT = (C.c_double * 16)()
    rc = _lib.load().pcp_icp_solve(_lib.f64arr(a), int(do_scale), dT)
    return rc, np.array(dT[:]).reshape(4, 4)


def get_rot_icp(ctx, src, temp, rmax, iters=20, do_scale=False, cell_size=0.0, src_dense=True,
                temp_dense=True):
    M = (C.c_double * 16)()
    err = C.c_float()
    ctx.check(ctx.lib.pcp_get_rot_icp(ctx.h, _ptr(src), src.shape[0], int(src_dense), _ptr(temp),
                                      temp.shape[0], int(temp_dense), M, float(rmax), int(iters),
                                      int(do_scale), float(cell_size), C.byref(err)))
    return float(err.value), np.array(M[:]).reshape(4, 4)
