"""Callers of the hot path restructured to batch: the reference's
per-point / per-frame loops around kNN / radius become one batched pcp_* call each.

  get_overlap_stamp(poses, stamps)        PointCloudClosure::get_overlap_stamp
                                          (point_cloud_closure.cpp:44-180): one batched
                                          radiusSearch(r = 10) over the trajectory, then the
                                          reference's first-passing-candidate scan of each
                                          sorted row and the segment grouping
  find_reliable(rots, load_cloud, thr)    find_reliable (main_blend.cpp:327-380): per frame the
                                          centre cloud's index and two batched
                                          find_cloud_nearest_point_in_kdtree reductions
                                          (pcp_nearest_query, one MIN over all queries)
"""
import math

import numpy as np
import torch

from . import ops

RAD2DEG = 57.29578  # macros.h:15


def _d_rots(poses, stamps):
    """The trajectory points of get_overlap_stamp (:46-79): position, stamp, heading (deg in
    [0, 360)), squared step; steps with distance_sqr <= 0.1 dropped."""
    out = []
    for i in range(len(poses) - 1):
        x, y, z = poses[i][0][3], poses[i][1][3], poses[i][2][3]
        dx, dy, dz = poses[i + 1][0][3] - x, poses[i + 1][1][3] - y, poses[i + 1][2][3] - z
        ang = math.atan2(dy, dx) * RAD2DEG
        dist = math.pow(dx, 2) + math.pow(dy, 2) + math.pow(dz, 2)
        if ang < 0:
            ang += 360.0
        if dist <= 0.1:
            continue
        out.append((x, y, z, int(stamps[i]), ang))
    return out


def _segments(pair_vec):
    """The segment grouping of get_overlap_stamp (:132-174)."""
    segs = []
    if not pair_vec:
        return segs
    base_start, frame_start = pair_vec[0]
    for i in range(1, len(pair_vec)):
        if abs(pair_vec[i][0] - pair_vec[i - 1][0]) > 10 or abs(pair_vec[i][1] - pair_vec[i - 1][1]) > 10:
            segs.append([base_start, pair_vec[i - 1][0], frame_start, pair_vec[i - 1][1]])
            base_start, frame_start = pair_vec[i]
    segs.append([base_start, pair_vec[-1][0], frame_start, pair_vec[-1][1]])
    for s in segs:
        if s[2] > s[3]:
            s[2], s[3] = s[3], s[2]
    return [tuple(s) for s in segs]


def _first_pair(pts, i, row):
    """The scan of one sorted radiusSearch row (:88-127): the first later, >= 6000 ms apart,
    same-heading (< 20 deg) neighbour within 1.5 m of the driving line."""
    cx, cy, _, cs, a1 = pts[i]
    for j in row:
        x2, y2, _, s2, a2 = pts[j]
        if s2 <= cs or abs(cs - s2) < 6000:
            continue
        if abs(a1 - a2) >= 20.0:
            continue
        avg = ((a1 + a2) / 2.0 - 90) / 180.0 * math.pi
        k = math.tan(avg)
        b = cy - k * cx
        if abs(0 - k * x2 + y2 - b) / math.sqrt(k * k + 1) > 1.5:
            continue
        return s2
    return None


def get_overlap_stamp(ctx, poses, stamps):
    """-> [(base_start, base_end, frame_start, frame_end)] stamps of the overlapping segments."""
    pts = _d_rots(poses, stamps)
    if not pts:
        return []
    xyz = torch.tensor([p[:3] for p in pts], dtype=torch.float64, device=ctx.device)
    ix = ops.GridIndex(ctx, xyz)
    offs, idx, _ = ops.radius(ix, xyz, 10.0)  # kd_tree.radiusSearch(cur_p, 10, ...) for every point
    offs, idx = offs.cpu().numpy(), idx.cpu().numpy()
    ix.close()
    pair_vec = []
    for i in range(len(pts)):
        s2 = _first_pair(pts, i, idx[offs[i]:offs[i + 1]])
        if s2 is not None:
            pair_vec.append((pts[i][3], s2))
    return _segments(pair_vec)


def find_reliable(ctx, rots, load_cloud, icp_threshold):
    """rots: list of dicts {matrix (4x4), stamp, icperr}; load_cloud(stamp) -> (n, 48) uint8 device
    cloud.  Returns the is_valid flags (main_blend.cpp:327-380, dis_threshold 0.06)."""
    valid = [False] * len(rots)
    for i in range(1, len(rots) - 1):
        e0, e1, e2 = rots[i - 1]["icperr"], rots[i]["icperr"], rots[i + 1]["icperr"]
        if not (e1 >= 0 and e1 <= icp_threshold and e0 >= 0 and e2 >= 0):
            continue
        left, right, centre = (load_cloud(rots[k]["stamp"]) for k in (i - 1, i + 1, i))
        ix = ops.GridIndex(ctx, centre)
        dis = []
        for cloud, (ma, mb) in ((left, (i - 1, i)), (right, (i, i + 1))):
            q, _ = ops.nearest_query(ix, cloud)
            # the default CloudItem when no query beats 9999 (x = y = z = 0, data[3] = 1)
            p = np.array([0.0, 0.0, 0.0, 1.0])
            if q >= 0:
                p = cloud[q].cpu().numpy().view(np.float64)[:4].copy()
            ta = np.asarray(rots[ma]["matrix"], dtype=np.float64) @ p
            tb = np.asarray(rots[mb]["matrix"], dtype=np.float64) @ p
            dis.append(math.pow(ta[0] - tb[0], 2) + math.pow(ta[1] - tb[1], 2) + math.pow(ta[2] - tb[2], 2))
        ix.close()
        if dis[0] < 0.06 and dis[1] < 0.06:
            valid[i] = True
    return valid


# ---------------------------------------------------------------- do_mul_frame_icp
def _frame_walk(line, start, step, valid_count, min_icp_threshold, stamp_file, stamps_out):
    """The front / back walks of do_mul_frame_icp (main_blend.cpp:684-745): collect frames from
    `start` outwards until valid_count consecutive frames have 0 < icp value < threshold.  The
    reference's consecutiveness tests differ by direction, and both are kept: walking back it
    is `(size_t)last_valid_index < size && last_valid_index != l + 1` (the unset -1 compares
    as SIZE_MAX), walking forward `last_valid_index >= 0 && last_valid_index != l - 1`; a
    gap resets k to 0 after the increment, so the frame that ends the gap does not count."""
    k, l, last = 0, start, -1
    n = len(line)
    while True:
        if (step < 0 and l < 0) or (step > 0 and l >= n):
            break
        v = float(np.float32(line[l]["icperr"]))  # const float icp_value = ..._value_icp
        if v > 0 and v < min_icp_threshold:
            k += 1
            gap = (last >= 0 and last < n and last != l + 1) if step < 0 else (last >= 0 and last != l - 1)
            if gap:
                k = 0
            last = l
        st = line[l]["stamp"]
        l += step
        if st in stamp_file:
            stamps_out.append((st, stamp_file[st]))
        if not k < valid_count:
            break


def _box_pad(ctx, cloud, pad):
    """getMinMax3D(cloud, PointT&, PointT&) (point_cloud_helper.h:22-57) widened by `pad`."""
    mn, mx = ops.minmax(ctx, cloud, True)
    return (mn[0] - pad, mn[1] - pad, mn[2] - pad), (mx[0] + pad, mx[1] + pad, mx[2] + pad)


def do_mul_frame_icp(ctx, line, stamp_file, start_index, end_index, grid, valid_count, min_icp_threshold,
                     is_do_sep_icp=False, is_mul_seg=False, is_shaft_filter=False, load_cloud=None):
    """do_mul_frame_icp (main_blend.cpp:641-931) on the device path.  line: the pose line, a list
    of dicts {stamp, matrix (4x4), icperr} (g_status._clouds_stamp_rot_line; matrices are
    updated in place, at the first entry of each stamp as get_cloud_rot_with_stamp does);
    stamp_file: stamp -> PCD path; grid: the CloudGrid map cache.  load_cloud(path) -> (n, 48)
    uint8 device records, or (records, is_dense) (default: pcd.load_pcd_ex, which reports
    is_dense as the reference's reader does); a plain tensor counts as dense when its xyz are
    all finite.  The joint frame's is_dense is the AND of the
    loaded clouds' (PointCloud::operator+=, point_cloud.h:130-147).  Returns (dis, rot) of
    the joint registration."""
    import torch
    from . import pcd as _pcd
    from . import segments as _seg
    if load_cloud is None:
        def load_cloud(path):
            arr, dense_f, _, _ = _pcd.load_pcd_ex(path)
            return torch.from_numpy(arr.view(np.uint8).reshape(-1, 48).copy()).to(ctx.device), dense_f
    frames = []  # (stamp, path) in frame_files order
    for i in range(start_index + 1, end_index):  # the frames between the two ends (:662-679)
        st = line[i]["stamp"]
        if st in stamp_file:
            frames.append((st, stamp_file[st]))
    _frame_walk(line, start_index, -1, valid_count, min_icp_threshold, stamp_file, frames)
    _frame_walk(line, end_index, +1, valid_count, min_icp_threshold, stamp_file, frames)
    loaded = [load_cloud(p) for _, p in frames]  # (:754-765)
    clouds = [c[0] if isinstance(c, tuple) else c for c in loaded]
    def _finite(rec):  # a plain tensor carries no flag: its is_dense is the data's finiteness
        xyz = rec.contiguous().view(torch.float64).reshape(-1, 6)[:, :3]  # any row / column slice
        return bool(torch.isfinite(xyz).all())
    dense = all(c[1] if isinstance(c, tuple) else _finite(c) for c in loaded)  # operator+= (point_cloud.h:143-146)
    frame = torch.cat(clouds) if clouds else torch.empty((0, 48), dtype=torch.uint8, device=ctx.device)
    frame = frame.clone()
    frame[:, 32:36] = torch.tensor([0, 0, 255, 0], dtype=torch.uint8, device=ctx.device)  # change_cloud_rgb 255,0,0
    frame = ops.remove_duplicate(ctx, frame, 0.04, is_dense=dense)
    if is_shaft_filter:
        frame = _seg.shaft_filter(ctx, frame)
    if not is_mul_seg:  # (:779-790): the map cache around the frames' box +- 30 m
        lo, hi = _box_pad(ctx, frame, 30.0)
        cache = grid.get_cloud_with_pos(lo, hi)
    else:  # get_grid_cloud(frame_cloud, frame_cloud, cache_cloud, 1.0) (:792): frame <- its matched part
        frame, cache = grid.get_grid_cloud_match(frame, 1.0)
    dis, rot = ops.get_rot_icp(ctx, cache, frame, 0.25, do_scale=True)  # get_rot_icp(cache, frame, rot, true)
    by_stamp = {}
    for i, e in enumerate(line):
        by_stamp.setdefault(e["stamp"], i)
    for (st, _), cloud in zip(frames, clouds):  # (:839-904)
        final = rot
        if is_do_sep_icp:
            moved = ops.transform(ctx, cloud, rot)
            lo, hi = _box_pad(ctx, moved, 3.0)
            cache_t = grid.get_cloud_with_pos(lo, hi)
            rot_split = np.eye(4)
            if cache_t.shape[0] > 0:
                _, rot_split = ops.get_rot_icp(ctx, cache_t, moved, 0.25, do_scale=False)
            final = rot_split @ rot
        if st in by_stamp:
            line[by_stamp[st]]["matrix"] = np.array(final)
    return dis, rot
