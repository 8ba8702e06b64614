"""CloudGrid (cloud_grid.cpp) -- the map cache behind every ICP target.

CPU: the C restatement (oracle/pcp_oracle.c ora_grid_*) against a line-by-line pure-Python
restatement of add_cloud_internal / get_cloud_with_pos / get_grid_cloud on small clouds
(parity unpinned otherwise: the reference has no test or fixture for CloudGrid).
GPU: libpcp's pcp_grid_* byte-exact against the C restatement: the greedy 4 cm
de-duplication per 1 m cell (including the (int) truncation that merges (-1, 1) into cell 0 and
incremental adds), the box query order, and get_grid_cloud's matching and push order."""
import math
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ctypes as ora  # noqa: E402


def scene(n, seed, span=6.0, dup=0.3):
    """Points around the origin (negative coordinates: the truncation quirk), a tall
    structure (cells with > 1.5 m of z) and near-duplicates (< 4 cm apart)."""
    rng = np.random.default_rng(seed)
    m = int(n * (1 - dup))
    xyz = np.empty((n, 3))
    xyz[:m, :2] = rng.uniform(-span, span, (m, 2))
    xyz[:m, 2] = rng.normal(0, 0.05, m)
    wall = rng.random(m) < 0.3
    xyz[:m][wall, 2] = rng.uniform(0, 4.0, wall.sum())
    src = rng.integers(0, m, n - m)
    xyz[m:] = xyz[src] + rng.uniform(-0.05, 0.05, (n - m, 3))
    perm = rng.permutation(n)
    return ora.make_cloud(xyz[perm], rgba=rng.integers(0, 2**31, n).astype(np.uint32),
                          stamp=np.arange(n, dtype=np.uint32))


class PyGrid:
    """cloud_grid.cpp restated line by line in Python (small inputs only)."""

    def __init__(self):
        self.cells = {}

    def add(self, cloud):
        for p in cloud:
            key = (int(p["x"]), int(p["y"]))
            if key not in self.cells:
                self.cells[key] = [p]
                continue
            keep = True
            for q in self.cells[key]:
                if abs(q["x"] - p["x"]) > 0.04 or abs(q["y"] - p["y"]) > 0.04 or abs(q["z"] - p["z"]) > 0.04:
                    continue
                d = np.float32((q["x"] - p["x"]) * (q["x"] - p["x"]) + (q["y"] - p["y"]) * (q["y"] - p["y"])
                               + (q["z"] - p["z"]) * (q["z"] - p["z"]))
                if float(d) < 0.04 * 0.04:
                    keep = False
                    break
            if keep:
                self.cells[key].append(p)

    def box(self, i0, i1, j0, j1):
        return [p for i in range(i0, i1) for j in range(j0, j1) for p in self.cells.get((i, j), [])]

    def match(self, src, dis):
        used, so, dst = {}, [], []
        for p in src:
            key = (int(p["x"]), int(p["y"]))
            cell = self.cells.get(key)
            if cell is None:
                continue
            zs = [q["z"] for q in cell]
            if max([np.finfo(np.float64).tiny] + zs) - min(zs) < 1.5:
                continue
            found = False
            for k, q in enumerate(cell):
                if abs(q["x"] - p["x"]) > dis or abs(q["y"] - p["y"]) > dis or abs(q["z"] - p["z"]) > dis:
                    continue
                found = True
                if k in used.setdefault(key, set()):
                    continue
                used[key].add(k)
                dst.append(q)
            if found:
                so.append(p)
        return so, dst


def recs(a):
    return np.asarray([r.tobytes() for r in a])


def test_oracle_grid_vs_python_restatement():
    c1, c2 = scene(3000, 1), scene(2000, 2)
    g, pg = ora.Grid(), PyGrid()
    for c in (c1, c2):
        g.add_cloud(c)
        pg.add(c)
    assert g.size == sum(len(v) for v in pg.cells.values())
    for (i0, i1, j0, j1) in [(-7, 7, -7, 7), (-2, 3, 0, 1), (0, 1, -1, 2)]:
        assert np.array_equal(recs(g.box(i0, i1, j0, j1)), recs(pg.box(i0, i1, j0, j1)))
    src = scene(800, 3)
    so, dst = g.match(src, 0.3)
    pso, pdst = pg.match(src, 0.3)
    assert len(dst) > 0 and np.array_equal(recs(so), recs(pso)) and np.array_equal(recs(dst), recs(pdst))


@pytest.mark.gpu
@pytest.mark.parametrize("n,span", [(20_000, 6.0), (400_000, 40.0)])
def test_gpu_grid_matches_oracle(n, span):
    import torch
    from pointcloudprocess_amd import cloudgrid, ops
    ctx = ops.Context(0)
    c1, c2 = scene(n, 11, span), scene(n // 2, 12, span)
    g, og = cloudgrid.CloudGrid(ctx), ora.Grid()
    for c in (c1, c2):  # two adds: the second one's points meet the first one's kept points
        g.add_cloud_internal(ops.cloud_to_device(c, ctx.device))
        og.add_cloud(c)
    assert g.size == og.size
    got = ops.cloud_to_host(g.get_grid_cloud())
    assert np.array_equal(recs(got), recs(og.points()))
    for mn, mx in [((-3.5, -2.2), (2.5, 4.0)), ((-span, -span), (span, span)), ((0.2, 0.7), (1.0, 1.0))]:
        got = ops.cloud_to_host(g.get_cloud_with_pos(mn, mx))
        exp = og.box(int(mn[0]), math.ceil(mx[0]), int(mn[1]), math.ceil(mx[1]))
        assert np.array_equal(recs(got), recs(exp)), (mn, mx)
    rot = np.eye(4)
    rot[0, 3], rot[1, 3] = -1.7, 2.9
    got = ops.cloud_to_host(g.get_cloud_with_pos_rot(rot, 3))
    assert np.array_equal(recs(got), recs(og.box(-1 - 3, -1 + 3, 2 - 3, 2 + 3)))
    src = scene(n // 4, 13, span)
    so, dst = g.get_grid_cloud_match(ops.cloud_to_device(src, ctx.device), 0.3)
    eso, edst = og.match(src, 0.3)
    assert len(edst) > 0
    assert np.array_equal(recs(ops.cloud_to_host(so)), recs(eso))
    assert np.array_equal(recs(ops.cloud_to_host(dst)), recs(edst))
    g.clear()
    assert g.size == 0
    g.close()
    ctx.close()
