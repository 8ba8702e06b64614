"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the pose-line composition (I4), the checker
of libpcp's pcp_pose_* (pointcloudprocess_amd/csrc/poses.cpp).  Parity pinned to the Eigen
formulas the reference calls (Eigen is not in the reference tree, so not run here):
  Affine3d(M).rotation()  -> polar factor U diag(1,1,sign det(UV^T)) V^T of the SVD
                             (Transform::computeRotationScaling, via numpy.linalg.svd)
  Quaterniond(R)          -> quaternionbase_assign_impl (trace > 0 / largest-diagonal branches)
  Identity().slerp(w, q)  -> QuaternionBase::slerp (the 1 - epsilon linear branch)
  toRotationMatrix, Translation3d * Quaterniond, Matrix4d::inverse.
References: main_blend.cpp:934-980, point_cloud_closure.cpp:185-276."""
import numpy as np


def polar_rotation(A):
    U, s, Vt = np.linalg.svd(A)
    x = -1.0 if np.linalg.det(U @ Vt) < 0 else 1.0
    U = U.copy()
    U[:, 2] *= x
    return U @ Vt


def quat_from_rot(m):
    q = np.zeros(4)  # x, y, z, w
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        s = np.sqrt(t + 1.0)
        q[3] = 0.5 * s
        s = 0.5 / s
        q[0] = (m[2, 1] - m[1, 2]) * s
        q[1] = (m[0, 2] - m[2, 0]) * s
        q[2] = (m[1, 0] - m[0, 1]) * s
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * s
        s = 0.5 / s
        q[3] = (m[k, j] - m[j, k]) * s
        q[j] = (m[j, i] + m[i, j]) * s
        q[k] = (m[k, i] + m[i, k]) * s
    return q


def slerp_identity(t, q):
    one = 1.0 - np.finfo(np.float64).eps
    d = q[3]
    if abs(d) >= one:
        s0, s1 = 1.0 - t, t
    else:
        th = np.arccos(abs(d))
        s0, s1 = np.sin((1.0 - t) * th) / np.sin(th), np.sin(t * th) / np.sin(th)
    if d < 0:
        s1 = -s1
    return s0 * np.array([0.0, 0.0, 0.0, 1.0]) + s1 * q


def rot_from_quat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def correction(L, length, k):
    A = L[:3, :3]
    R = polar_rotation(A)
    q = quat_from_rot(R)
    eps = A @ np.linalg.inv(R) - np.eye(3)
    w = k / (length - 1)
    E = np.eye(4)
    E[:3, :3] = (np.eye(3) + w * eps) @ rot_from_quat(slerp_identity(w, q))
    E[:3, 3] = w * L[:3, 3]
    return E


def interpolate(rots, start, end):
    rots = rots.copy()
    base = rots[start].copy()
    L = rots[end] @ np.linalg.inv(base)
    n = end - start + 1
    for i in range(start, end + 1):
        rots[i] = correction(L, n, i - start) @ base
    return rots


def lum_elch(rots, start, end, loop):
    rots = rots.copy()
    n = end - start + 1
    for i in range(start, end + 1):
        rots[i] = correction(loop, n, i - start) @ rots[i]
    return rots


def loop_closure(ori, ori_stamps, opt, opt_stamps, window=400):
    ori = ori.copy()
    idx = {int(s): i for i, s in reversed(list(enumerate(ori_stamps)))}
    s0, s1 = idx.get(int(opt_stamps[0]), -1), idx.get(int(opt_stamps[-1]), -1)
    if s0 < 0 or s1 < 0 or s1 - s0 + 1 != len(opt):
        return False, ori
    pair = opt[0] @ np.linalg.inv(ori[s0])
    endT = opt[-1] @ np.linalg.inv(ori[s1])
    ori = lum_elch(ori, max(s0 - window + 1, 0), s0, pair)
    ori[s0:s1 + 1] = opt
    for i in range(s1 + 1, len(ori)):
        ori[i] = endT @ ori[i]
    return True, ori
