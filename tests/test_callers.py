"""Batched callers against per-point restatements of the reference's
loops over the oracle kd-tree (FLANN-order radiusSearch / nearestKSearch)."""
import math
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ctypes as ora  # noqa: E402
from pointcloudprocess_amd import callers  # noqa: E402


def trajectory(seed):
    """A drive around a block twice (the second lap overlaps the first, 90 s later)."""
    rng = np.random.default_rng(seed)
    poses, stamps = [], []
    t = 1_000_000
    for lap in range(2):
        for k in range(400):
            s = k / 400.0 * 4
            side, f = int(s), s - int(s)
            corners = [(0, 0), (120, 0), (120, 80), (0, 80), (0, 0)]
            (x0, y0), (x1, y1) = corners[side], corners[side + 1]
            T = np.eye(4)
            T[0, 3] = x0 + f * (x1 - x0) + rng.normal(0, 0.2) + 0.3 * lap
            T[1, 3] = y0 + f * (y1 - y0) + rng.normal(0, 0.2)
            T[2, 3] = rng.normal(0, 0.05)
            poses.append(T)
            stamps.append(t)
            t += 100 + int(rng.integers(0, 5))
        t += 90_000
    return np.array(poses), np.array(stamps, dtype=np.uint64)


def overlap_reference(poses, stamps):
    pts = callers._d_rots(poses, stamps)
    tree = ora.KdTree(np.array([p[:3] for p in pts]))
    pair_vec = []
    for i in range(len(pts)):
        row, _ = tree.radius(np.array(pts[i][:3]), 10.0)
        s2 = callers._first_pair(pts, i, row)
        if s2 is not None:
            pair_vec.append((pts[i][3], s2))
    return callers._segments(pair_vec)


def test_overlap_rows_oracle_self_consistent():
    poses, stamps = trajectory(1)
    segs = overlap_reference(poses, stamps)
    assert len(segs) >= 1 and all(s[0] <= s[1] and s[2] <= s[3] for s in segs)


@pytest.mark.gpu
def test_gpu_get_overlap_stamp(ctx=None):
    from pointcloudprocess_amd import ops
    ctx = ops.Context(0)
    poses, stamps = trajectory(2)
    assert callers.get_overlap_stamp(ctx, poses, stamps) == overlap_reference(poses, stamps)
    ctx.close()


@pytest.mark.gpu
def test_gpu_find_reliable():
    import torch
    from pointcloudprocess_amd import ops, synth
    ctx = ops.Context(0)
    base = synth.street_scene(60_000, 81, extent=(40.0, 40.0)).double().numpy()
    rng = np.random.default_rng(5)
    clouds, rots = {}, []
    for i in range(8):
        T = np.eye(4)
        T[:3, 3] = [0.01 * i, 0.0, 0.0]
        sel = rng.choice(len(base), 20_000, replace=False)
        clouds[1000 + i] = ora.make_cloud(base[sel] + rng.normal(0, 0.002, (20_000, 3)))
        rots.append({"matrix": T, "stamp": 1000 + i, "icperr": [0.05, 0.05, 0.5, 0.05, -1, 0.05, 0.05, 0.05][i]})
    rots[6]["matrix"] = rots[6]["matrix"].copy()
    rots[6]["matrix"][0, 3] += 1.0  # a jump: frames 5..7 unreliable
    dev = {s: ops.cloud_to_device(c, ctx.device) for s, c in clouds.items()}
    got = callers.find_reliable(ctx, rots, lambda s: dev[s], 0.13)
    # the reference's loops on the oracle kd-tree
    exp = [False] * len(rots)
    for i in range(1, len(rots) - 1):
        e0, e1, e2 = rots[i - 1]["icperr"], rots[i]["icperr"], rots[i + 1]["icperr"]
        if not (0 <= e1 <= 0.13 and e0 >= 0 and e2 >= 0):
            continue
        c = clouds[rots[i]["stamp"]]
        tree = ora.KdTree(np.stack([c["x"], c["y"], c["z"]], 1))
        dis = []
        for nb, (a, b) in ((clouds[rots[i - 1]["stamp"]], (i - 1, i)), (clouds[rots[i + 1]["stamp"]], (i, i + 1))):
            _, d2 = tree.knn(np.stack([nb["x"], nb["y"], nb["z"]], 1), 1)
            best, mix = -1, 9999.0
            for j in range(len(nb)):
                if d2[j, 0] < mix:
                    mix, best = d2[j, 0], j
            p = np.array([nb["x"][best], nb["y"][best], nb["z"][best], 1.0])
            ta, tb = rots[a]["matrix"] @ p, rots[b]["matrix"] @ p
            dis.append(sum(math.pow(ta[k] - tb[k], 2) for k in range(3)))
        exp[i] = dis[0] < 0.06 and dis[1] < 0.06
    assert got == exp and any(exp) and not all(exp[1:-1])
    ctx.close()
