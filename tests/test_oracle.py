"""Pin the CPU oracle before trusting it (CPU only, no GPU).

* the reference's own known-answer tests (tests/golden/kat_*.json, generated from
  main_test.cpp:126-188 semantics by tests/golden/make_golden.py);
* exact kNN / radius against scipy.spatial.cKDTree and numpy brute force;
* VoxelGrid quirks (truncation, float-cast averaging, rgb packing) against an
  independent numpy restatement;
* 3x3 eigen against numpy.linalg.eigh; ICP recovers a known rigid motion.
"""
import json
import os

import numpy as np
import pytest
from scipy.spatial import cKDTree

import oracle_ctypes as ora

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_kat_kd_tree():
    g = load_golden("kat_kd_tree.json")
    t = ora.KdTree(np.array(g["cloud_xyz"]))
    idx, d2 = t.knn(np.array(g["query"]), g["k"])
    assert idx[0].tolist() == g["expected_indices"]
    assert d2[0].tolist() == g["expected_sqr_distances"]  # bit-exact


def test_kat_voxel_grid():
    g = load_golden("kat_voxel_grid.json")
    cloud = ora.make_cloud(np.array(g["cloud_xyz"]))
    out, vidx = ora.voxel_filter(cloud, tuple(g["leaf"]))
    assert len(out) == len(g["expected"])
    for o, v, e in zip(out, vidx, g["expected"]):
        assert int(v) == e["voxel_idx"]
        assert [o["x"], o["y"], o["z"]] == e["xyz"]  # bit-exact
    assert out[0]["x"] == 0.4090909111228856  # float-cast averaging (concatenate.h:153)


@pytest.mark.parametrize("k", [1, 8, 20])
def test_knn_vs_scipy(k):
    rng = np.random.default_rng(7 + k)
    pts = rng.uniform(-50, 50, size=(20000, 3)).astype(np.float32).astype(np.float64)
    q = rng.uniform(-50, 50, size=(2000, 3)).astype(np.float32).astype(np.float64)
    t = ora.KdTree(pts)
    idx, d2 = t.knn(q, k)
    ref = cKDTree(pts)
    rd, ri = ref.query(q, k=k)
    ri = ri.reshape(len(q), k)
    assert np.array_equal(idx, ri)
    # distances: L2_Simple accumulation order ((0+d0^2)+d1^2)+d2^2
    dd = q[:, None, :] - pts[idx]
    exp = (dd[..., 0] * dd[..., 0] + dd[..., 1] * dd[..., 1]) + dd[..., 2] * dd[..., 2]
    assert np.array_equal(d2, exp)


def test_knn_brute_force_ties():
    # integer lattice => many exact ties; order must be (d2, index) lexicographic
    g = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(6), indexing="ij"), -1)
    pts = g.reshape(-1, 3).astype(np.float64)
    t = ora.KdTree(pts)
    q = np.array([[2.0, 2.0, 2.0], [0.5, 0.5, 0.5], [2.5, 1.0, 4.0]])
    idx, d2 = t.knn(q, 27)
    for i in range(len(q)):
        dd = ((q[i] - pts) ** 2).sum(1)
        order = np.lexsort((np.arange(len(pts)), dd))[:27]
        assert idx[i].tolist() == order.tolist()


def test_knn_nonfinite_and_indices():
    pts = np.array([[0, 0, 0], [np.nan, 0, 0], [1, 0, 0], [2, 0, 0], [np.inf, 1, 1]], float)
    t = ora.KdTree(pts)
    assert t.size == 3
    idx, d2 = t.knn(np.zeros(3), 5)  # k clamped to 3, padded with -1
    assert idx[0].tolist() == [0, 2, 3, -1, -1]
    t2 = ora.KdTree(pts, indices=[3, 1, 2])
    idx, _ = t2.knn(np.zeros(3), 2)
    assert idx[0].tolist() == [2, 3]


def test_radius_vs_scipy():
    rng = np.random.default_rng(3)
    pts = rng.uniform(0, 10, size=(5000, 3))
    t = ora.KdTree(pts)
    ref = cKDTree(pts)
    for q in rng.uniform(0, 10, size=(50, 3)):
        idx, d2 = t.radius(q, 1.0)
        exp = sorted(ref.query_ball_point(q, 1.0 - 1e-12))
        assert sorted(idx.tolist()) == exp
        assert np.all(np.diff(d2) >= 0)
        idx5, _ = t.radius(q, 1.0, max_nn=5)
        assert idx5.tolist() == idx[:5].tolist()


def numpy_voxel(xyz, rgba, stamp, leaf):
    """Independent numpy restatement of voxel_grid.h:811-1056 for finite clouds."""
    inv = 1.0 / np.asarray(leaf, float)
    mn = xyz.min(0)
    mx = np.maximum(xyz.max(0), np.finfo(float).tiny)
    min_b = np.trunc(mn * inv).astype(np.int64)
    max_b = np.trunc(mx * inv).astype(np.int64)
    div = max_b - min_b + 1
    ijk = np.trunc(xyz * inv - min_b).astype(np.int64)
    idx = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]) & 0xFFFFFFFF
    order = np.lexsort((np.arange(len(xyz)), idx))
    s_idx = idx[order]
    starts = np.flatnonzero(np.r_[True, s_idx[1:] != s_idx[:-1]])
    fields = np.c_[xyz.astype(np.float32).astype(np.float64),
                   rgba.astype(np.float32).astype(np.float64),
                   stamp.astype(np.float32).astype(np.float64),
                   (rgba >> 16) & 0xFF, (rgba >> 8) & 0xFF, rgba & 0xFF][order]
    out = []
    for a, b in zip(starts, np.r_[starts[1:], len(order)]):
        c = fields[a].copy()
        for r in range(a + 1, b):
            c = c + fields[r]
        out.append((s_idx[a], c / (b - a)))
    return out


def test_voxel_random_vs_numpy():
    rng = np.random.default_rng(11)
    xyz = rng.uniform(-3, 5, size=(4000, 3)).astype(np.float32).astype(np.float64)
    rgba = rng.integers(0, 2**32, size=4000, dtype=np.uint64).astype(np.uint32)
    stamp = rng.integers(0, 2**31, size=4000, dtype=np.uint64).astype(np.uint32)
    cloud = ora.make_cloud(xyz, rgba, stamp)
    out, vidx = ora.voxel_filter(cloud, (0.5, 0.7, 0.3))
    exp = numpy_voxel(xyz, rgba, stamp, (0.5, 0.7, 0.3))
    assert len(out) == len(exp)
    for o, v, (ei, c) in zip(out, vidx, exp):
        assert int(v) == int(ei)
        assert (o["x"], o["y"], o["z"]) == (c[0], c[1], c[2])
        assert o["stamp_id"] == np.uint32(c[4])
        r, g, b = np.float32(c[5]), np.float32(c[6]), np.float32(c[7])
        assert o["rgba"] == (int(r) << 16) | (int(g) << 8) | int(b)


def test_voxel_truncation_slab():
    # min < 0: truncation makes the first slab two leaves wide
    xyz = np.array([[-0.9, 0, 0], [0.9, 0, 0], [1.1, 0, 0]], float)
    out, vidx = ora.voxel_filter(ora.make_cloud(xyz), 1.0)
    assert len(out) == 2 and out[0]["x"] == np.float64((np.float32(-0.9) + np.float32(0.9)) / 2)


def test_voxel_nonfinite_and_empty():
    xyz = np.array([[0, 0, 0], [np.nan, 1, 1], [0.1, 0.1, 0.1]], float)
    out, _ = ora.voxel_filter(ora.make_cloud(xyz), 1.0, is_dense=False)
    assert len(out) == 1
    out, _ = ora.voxel_filter(ora.make_cloud(np.zeros((0, 3))), 1.0)
    assert len(out) == 0


def test_eigen_sym3_vs_numpy():
    rng = np.random.default_rng(5)
    lib = ora.load()
    for _ in range(200):
        a = rng.normal(size=(3, 3))
        A = np.ascontiguousarray(a @ a.T)
        ev, E = np.zeros(3), np.zeros(9)
        lib.ora_eigen_sym3(A.ctypes.data, ev.ctypes.data, E.ctypes.data)
        E = E.reshape(3, 3)
        w, V = np.linalg.eigh(A)
        assert np.allclose(ev, w[::-1], rtol=1e-12, atol=1e-12)
        for i in range(3):
            assert np.allclose(A @ E[i], ev[i] * E[i], atol=1e-10)


def test_plane_h_points_flat():
    rng = np.random.default_rng(2)
    xy = rng.uniform(-1, 1, size=(32, 2))
    pts = np.c_[xy, 0.5 * xy[:, 0] + 0.25 * xy[:, 1] + 3.0]
    out = ora.normals_knn(pts, 32)
    n = np.array([-0.5, -0.25, 1.0]) / np.linalg.norm([-0.5, -0.25, 1.0])
    got = np.array([out["normal_x"][0], out["normal_y"][0], out["normal_z"][0]])
    assert abs(abs(got @ n) - 1) < 1e-6
    assert got[2] > 0  # largest component positive
    assert abs(out["curvature"][0]) < 1e-6


def test_icp_recovers_motion():
    rng = np.random.default_rng(1)
    # gentle terrain so point-to-point ICP is well conditioned
    xy = rng.uniform(-10, 10, size=(20000, 2))
    tgt = np.c_[xy, np.sin(xy[:, 0] * 0.7) + 0.5 * np.cos(xy[:, 1] * 0.9)].astype(np.float32)
    ang = np.deg2rad(1.0)
    R = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
    t = np.array([0.05, -0.03, 0.02])
    q = ((tgt.astype(np.float64) - t) @ R).astype(np.float32)  # q = R^T (p - t)
    err, T = ora.icp(tgt, q, np.eye(4), rmax=0.5, iters=40)
    assert err >= 0 and err < 1e-3
    assert np.allclose(T[:3, :3], R, atol=1e-4)
    assert np.allclose(T[:3, 3], t, atol=1e-3)


def test_knn_lod_contract():
    rng = np.random.default_rng(9)
    xyz = rng.uniform(100, 110, size=(3000, 3))
    cloud = ora.make_cloud(xyz)
    q = xyz[17] + 1e-3
    idx, d2 = ora.knn_lod(cloud, q, 4)
    assert idx[0] == 17
    exact = np.argsort(((xyz - q) ** 2).sum(1))[:4]
    assert set(idx.tolist()) <= set(exact.tolist()) | {-1}


def test_near_face_cloud_needs_the_sequential_fold():
    """Why remove_duplicate needs compute3DCentroid's exact sequential fold: on a cloud with
    points within 1e-12 m of voxel faces, a blocked (tree-order) centroid changes the output
    (tests/test_gpu_cloud.py::test_remove_duplicate_near_faces uses this cloud)."""
    import test_gpu_cloud as tg
    c = tg._near_face_cloud(200_000, 0.04, 17)
    xyz = np.stack([c["x"], c["y"], c["z"]], 1)
    blocked = np.append(xyz.reshape(-1, 1000, 3).sum(axis=1).sum(axis=0) / len(xyz), 0.0)
    e = ora.remove_duplicate(c, 0.04)
    e2 = ora.remove_duplicate_c(c, 0.04, blocked)
    assert len(e) != len(e2) or e.tobytes() != e2.tobytes()


def test_rpca_oracle_robust_and_deterministic():
    """F3 restated (ora_rpca, calculate_feature.cpp:208-368): on a noisy plane with 10 %
    outliers the robust normal stays on the plane's normal where the plain PCA (F1) tilts,
    the draws are a pure function of (seed, point, iteration, slot), and N <= 3 rows give
    {0, 0, 0, curvature 1} (:353-361)."""
    rng = np.random.default_rng(5)
    n = 3000
    xyz = np.c_[rng.uniform(-1, 1, (n, 2)), rng.normal(0, 1e-3, n)]
    out_i = rng.choice(n, n // 10, replace=False)
    xyz[out_i, 2] += rng.uniform(0.05, 0.2, len(out_i))
    _, idx = cKDTree(xyz).query(xyz, k=20)
    idx = idx.astype(np.int32)
    a = ora.rpca(xyz, idx, seed=7)
    b = ora.rpca(xyz, idx, seed=7)
    assert a.tobytes() == b.tobytes()
    inl = np.setdiff1d(np.arange(n), out_i)
    nz_r = np.abs(a["normal_z"][inl])
    f1 = ora.normals_knn(xyz, 20)
    nz_p = np.abs(f1["normal_z"][inl])
    assert np.median(nz_r) > 0.999 and nz_r.mean() > nz_p.mean()
    assert (a["point_id"] == np.arange(n)).all()
    short = idx.copy()
    short[:5, 3:] = -1
    c = ora.rpca(xyz, short, seed=7)
    assert (c["normal_x"][:5] == 0).all() and (c["curvature"][:5] == 1.0).all()
    assert ora.load().ora_rpca_draw(1, 2, 3, 0) != ora.load().ora_rpca_draw(1, 2, 3, 1)
