"""I4 pose lines (host-only, libpcp pcp_pose_*): against the numpy restatement of the Eigen
formulas (oracle/poses_oracle.py), plus the reference's invariants (weight 0 keeps the first
frame, weight 1 applies the whole correction, loop closure splices the optimised span)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import poses_oracle as ora  # noqa: E402
from pointcloudprocess_amd import poses  # noqa: E402


def rigid(rng, ang=0.05, tr=1.0, scale=1.0):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    th = rng.uniform(-ang, ang)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    T = np.eye(4)
    T[:3, :3] = scale * (np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K)
    T[:3, 3] = rng.uniform(-tr, tr, 3)
    return T


def line(rng, n):
    rots = np.empty((n, 4, 4))
    T = np.eye(4)
    for i in range(n):
        T = rigid(rng, 0.02, 2.0) @ T
        T[:3, 3] += [5.0 * i, 0.3 * i, 0.0]
        rots[i] = T
    return rots


@pytest.mark.parametrize("seed,scale", [(1, 1.0), (2, 1.0005), (3, 0.999)])
def test_interpolate_matches_oracle(seed, scale):
    rng = np.random.default_rng(seed)
    rots = line(rng, 40)
    rots[30] = rigid(rng, 0.3, 3.0, scale) @ rots[30]  # a jump to interpolate over (ICP with do_scale)
    exp = ora.interpolate(rots, 5, 30)
    got = poses.interpolate(rots.copy(), 5, 30)
    assert np.abs(got - exp).max() < 1e-9
    assert np.array_equal(got[:5], rots[:5]) and np.array_equal(got[31:], rots[31:])
    assert np.abs(got[5] - rots[5]).max() < 1e-12  # weight 0: the base frame itself
    assert np.abs(got[30] - rots[30]).max() < 1e-9  # weight 1: the end frame's pose


def test_lum_elch_matches_oracle():
    rng = np.random.default_rng(4)
    rots = line(rng, 50)
    loop = rigid(rng, 0.2, 1.5)
    exp = ora.lum_elch(rots, 10, 45, loop)
    got = poses.lum_elch(rots.copy(), 10, 45, loop)
    assert np.abs(got - exp).max() < 1e-9
    assert np.abs(got[45] - loop @ rots[45]).max() < 1e-9  # the last frame gets the whole loop
    # the slerp branch for a near-identity loop (|q.w| >= 1 - eps: linear weights)
    got2 = poses.lum_elch(rots.copy(), 0, 49, np.eye(4))
    assert np.abs(got2 - rots).max() < 1e-12


def test_loop_closure_matches_oracle():
    rng = np.random.default_rng(5)
    ori = line(rng, 600)
    stamps = np.arange(1000, 1600, dtype=np.uint64)
    opt = np.stack([rigid(rng, 0.01, 0.2) @ ori[i] for i in range(450, 480)])
    ok_e, exp = ora.loop_closure(ori, stamps, opt, stamps[450:480])
    got = ori.copy()
    ok = poses.loop_closure(got, stamps, opt, stamps[450:480])
    assert ok and ok_e
    assert np.abs(got - exp).max() < 1e-9
    assert np.array_equal(got[450:480], opt)
    # a stamp that is not in the line: the reference returns false and leaves it untouched
    got = ori.copy()
    assert not poses.loop_closure(got, stamps, opt, np.arange(5000, 5030, dtype=np.uint64))
    assert np.array_equal(got, ori)
