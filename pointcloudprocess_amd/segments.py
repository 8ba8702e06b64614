"""Plane segmentation by region growing and the static.cpp filters
built on it.

  region_growing(index, xyz, props, distance_t, cosfa_t)
        TreeExtration::region_growning (extraction_tree.cpp:66-272, live body :177-271) through
        pcp_region_growing: the 50-NN graph and the plane-distance edge test on the GPU, then
        the reference's sequential seed walk replayed on the host (segments.hip).
  point_segment(ctx, cloud)     static.cpp:8-21: kNN(20) -> rpca planes -> region growing
  tree_filter / shaft_filter / ground_filter   static.cpp:24-80

`cloud` is an (n, 3) float64 device tensor or (n, 48) uint8 AoS48 records (PointXYZRGBA);
the filters return the kept rows of that tensor in the reference's push order.
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import ops
from .ops import _ptr, _qstride

# point_segment's constants (static.cpp:9-14); radius / radius_in_growning are unused there
COSFA_T = 0.940
DISTANCE_T = 0.5
PR = 0.99
EPI = 0.5
KNN_RPCA = 20  # calculate_feature.cpp:233


@dataclass
class Segments:
    """vector<PlanSegment>: segment s holds points[offsets[s]:offsets[s+1]] in push order; its
    plane is its seed point's (normal_x/y/z and (float)Distance, extraction_tree.cpp:254-257)."""
    offsets: np.ndarray   # int64 (n_seg + 1)
    points: np.ndarray    # int32
    seeds: np.ndarray     # int32 (n_seg)
    planes: np.ndarray    # float32 (n_seg, 4): normal_x, normal_y, normal_z, Distance

    def __len__(self):
        return len(self.seeds)

    def point_ids(self, s):
        return self.points[self.offsets[s]:self.offsets[s + 1]]


def region_growing(index, xyz, props, distance_t=DISTANCE_T, cosfa_t=COSFA_T):
    """TreeExtration::region_growning.  props: (n, 48) uint8 device LAS_POINT_PROPERTY records
    (ops.normals_rpca); their segment_id is rewritten in place."""
    ctx = index.ctx
    n = xyz.shape[0]
    if props.shape[0] != n:
        raise ValueError("one LAS_POINT_PROPERTY per cloud point expected")
    offs = np.zeros(n + 1, np.int64)
    pts = np.empty(max(n, 1), np.int32)
    seeds = np.empty(max(n, 1), np.int32)
    nseg = C.c_int64()
    ctx.check(ctx.lib.pcp_region_growing(ctx.h, index.h, _ptr(xyz), _qstride(xyz), n, _ptr(props),
                                         float(distance_t), float(cosfa_t), offs.ctypes.data, pts.ctypes.data,
                                         seeds.ctypes.data, C.byref(nseg)))
    ns = nseg.value
    seeds = seeds[:ns].copy()
    planes = np.zeros((ns, 4), np.float32)
    if ns:
        rec = props[torch.from_numpy(seeds.astype(np.int64)).to(props.device)].cpu().numpy()
        rec = rec.view(ops.POINT_PROPERTY).reshape(ns)
        planes[:, 0], planes[:, 1], planes[:, 2] = rec["normal_x"], rec["normal_y"], rec["normal_z"]
        planes[:, 3] = rec["distance"].astype(np.float32)
    return Segments(offs[:ns + 1].copy(), pts[:offs[ns]].copy(), seeds, planes)


def point_segment(ctx, cloud, seed=0):
    """static.cpp:8-21.  Returns (Segments, props)."""
    index = ops.GridIndex(ctx, cloud)
    k = min(KNN_RPCA, max(index.size, 1))
    knn_idx, _ = ops.knn(index, cloud, k)
    props = ops.normals_rpca(ctx, cloud, knn_idx, PR, EPI, seed)
    return region_growing(index, cloud, props, DISTANCE_T, COSFA_T), props


def _gather(cloud, ids):
    return cloud[torch.from_numpy(np.asarray(ids, np.int64)).to(cloud.device)]


def tree_filter(ctx, cloud, seed=0):
    """static.cpp:24-36: the points of every segment with more than 50 points."""
    segs, _ = point_segment(ctx, cloud, seed)
    keep = [segs.point_ids(s) for s in range(len(segs)) if segs.offsets[s + 1] - segs.offsets[s] > 50]
    return _gather(cloud, np.concatenate(keep) if keep else np.empty(0, np.int64))


def shaft_filter(ctx, cloud, seed=0):
    """static.cpp:37-52: the points of every segment with |normal_z| < 0.30."""
    segs, _ = point_segment(ctx, cloud, seed)
    keep = [segs.point_ids(s) for s in range(len(segs)) if abs(float(segs.planes[s, 2])) < 0.30]
    return _gather(cloud, np.concatenate(keep) if keep else np.empty(0, np.int64))


def ground_filter(ctx, cloud, seed=0):
    """static.cpp:55-79: every point not in a segment with |normal_z| > 0.9, in index order."""
    segs, _ = point_segment(ctx, cloud, seed)
    ground = np.zeros(cloud.shape[0], bool)
    for s in range(len(segs)):
        if abs(float(segs.planes[s, 2])) > 0.9:
            ground[segs.point_ids(s)] = True
    return _gather(cloud, np.nonzero(~ground)[0])
