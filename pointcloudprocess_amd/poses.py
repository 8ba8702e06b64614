"""I4: pose lines around the ICP loop (host-only; libpcp's pcp_pose_* C-ABI).

A pose line is an (n, 4, 4) float64 array of frame poses, as CloudStampRot::_rot
(cloud_stamp_rot.h:7-39) along the trajectory; stamps are uint64.
  interpolate(rots, start, end)        do_transform_interpolation (main_blend.cpp:934-980)
  lum_elch(rots, start, end, loop)     PointCloudClosure::do_lum_elch (point_cloud_closure.cpp:194-233)
  loop_closure(ori, ori_stamps, opt, opt_stamps, window=400)
                                       PointCloudClosure::do_loop_closure (:235-276)
All three update the array in place (as the reference updates the vector) and return it.
"""
import ctypes as C

import numpy as np

from . import _lib


def _rots(a):
    a = np.asarray(a)
    if a.dtype != np.float64 or not a.flags.c_contiguous or a.ndim != 3 or a.shape[1:] != (4, 4):
        raise ValueError("pose line must be a C-contiguous (n, 4, 4) float64 array")
    return a


def interpolate(rots, start, end):
    r = _rots(rots)
    _lib.check(_lib.load().pcp_pose_interpolate(r.ctypes.data, len(r), int(start), int(end)))
    return r


def lum_elch(rots, start, end, loop):
    r = _rots(rots)
    L = np.ascontiguousarray(loop, dtype=np.float64).reshape(16)
    _lib.check(_lib.load().pcp_pose_lum_elch(r.ctypes.data, len(r), int(start), int(end), L.ctypes.data))
    return r


def loop_closure(ori, ori_stamps, opt, opt_stamps, window=400):
    """False (ori untouched) where the reference returns false: a stamp not found or a span
    length mismatch (point_cloud_closure.cpp:240-251)."""
    o = _rots(ori)
    p = np.ascontiguousarray(opt, dtype=np.float64)
    so = np.ascontiguousarray(ori_stamps, dtype=np.uint64)
    sp = np.ascontiguousarray(opt_stamps, dtype=np.uint64)
    rc = _lib.load().pcp_pose_loop_closure(o.ctypes.data, so.ctypes.data, len(o), p.ctypes.data, sp.ctypes.data,
                                           len(p), int(window))
    if rc == _lib.PCP_OK:
        return True
    if rc == -1:
        return False
    _lib.check(rc)
