"""GPU parity of the cloud passes (MI355X) against the oracle.

V2 getMinMax3D, I2 transformPointCloud, V3 VoxelGrid::applyFilter: BIT-EXACT (every byte
of every 48-byte output record, plus the u32 voxel index), including the reference KAT
(tests/golden/kat_voxel_grid.json, main_test.cpp:126-154) and the int32 wrap of the
linear voxel index.  I3 compute3DCentroid: BIT-EXACT against the reference's sequential
left fold (fold.hip's exact chunk-map scan), on adversarial inputs (sums through zero, huge
offsets, half-ulp ties, mixed magnitudes, NaN/Inf).  V4 remove_duplicate: every byte equal
to the sequential-centroid oracle, including points within 1e-12 of a voxel face.
I1 get_rot_icp: pose within 1e-5 (north_star tolerance; ICP is "parity unpinned"), dense and
non-dense inputs.
"""
import json
import os

import numpy as np
import pytest
import torch

import oracle_ctypes as ora

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


def _rand_cloud(n, seed, half=10.0, offset=(0.0, 0.0, 0.0), nan_every=0):
    rng = np.random.default_rng(seed)
    xyz = rng.uniform(-half, half, (n, 3)).astype(np.float32).astype(np.float64) + np.asarray(offset)
    if nan_every:
        xyz[::nan_every] = np.nan
    rgba = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    stamp = rng.integers(0, 2**20, n).astype(np.uint32)
    c = ora.make_cloud(xyz, rgba, stamp)
    c["w"] = rng.uniform(0.5, 1.5, n)
    return c


def _same_bytes(a, b):
    return np.ascontiguousarray(a).view(np.uint8).tobytes() == np.ascontiguousarray(b).view(np.uint8).tobytes()


@pytest.mark.parametrize("dense", [True, False])
def test_minmax(ctx, dense):
    from pointcloudprocess_amd import ops
    c = _rand_cloud(100_000, 1, nan_every=0 if dense else 37)
    mn, mx = ops.minmax(ctx, ops.cloud_to_device(c, ctx.device), is_dense=dense)
    emn, emx = ora.minmax(c, is_dense=dense)
    if dense:
        return  # NaN propagation under is_dense is the reference's undefined case
    assert np.array_equal(mn, emn) and np.array_equal(mx, emx)


def test_minmax_dbl_min_quirk(ctx):
    from pointcloudprocess_amd import ops
    c = _rand_cloud(1000, 2, half=1.0, offset=(-5.0, 3.0, -7.0))  # x and z all negative
    mn, mx = ops.minmax(ctx, ops.cloud_to_device(c, ctx.device))
    emn, emx = ora.minmax(c)
    assert np.array_equal(mn, emn) and np.array_equal(mx, emx)
    assert mx[0] == np.finfo(np.float64).tiny and mx[2] == np.finfo(np.float64).tiny


def _fold_cases():
    """(name, xyz, is_dense): inputs that stress the exact fold (fold.hip)."""
    rng = np.random.default_rng(11)
    cases = []
    n = 1_000_003
    # survey-scale offsets (UTM-like): long runs inside one binade -> chunk maps
    cases.append(("utm", rng.uniform(-50, 50, (n, 3)) + np.array([431_250.5, 4_412_020.25, 35.0]), True))
    # zero-mean: the running sums wander through 0 and across many binades
    cases.append(("zero_mean", rng.uniform(-100, 100, (n, 3)), True))
    # magnitudes from 1e-12 to 1e3 with random signs: rounding in every add
    mag = 10.0 ** rng.uniform(-12, 3, (n, 3))
    cases.append(("mixed_mag", mag * rng.choice([-1.0, 1.0], (n, 3)), True))
    # half-ulp ties: sum ~2^40 (u = 2^-12), addends odd multiples of 2^-13
    t = (2 * rng.integers(-2**20, 2**20, (n, 3)) + 1) * 2.0 ** -13
    t[0] = 2.0 ** 40
    cases.append(("ties", t, True))
    # float32-representable street-scene values (what C3/C4 clouds hold)
    cases.append(("f32", (rng.uniform(0, 200, (n, 3)).astype(np.float32)).astype(np.float64), True))
    # non-finite points skipped (!is_dense) and propagated (is_dense)
    bad = rng.uniform(-10, 10, (300_001, 3)) + 1000.0
    bad[::97, 0] = np.nan
    bad[5::131, 2] = np.inf
    bad[7::173, 1] = -np.inf
    cases.append(("nonfinite_skip", bad, False))
    cases.append(("nonfinite_dense", bad, True))
    # sizes around the chunk (2048) and a -0.0 first point
    for m in (1, 2, 2047, 2048, 2049, 4097):
        x = rng.uniform(-1, 1, (m, 3))
        x[0] = -0.0
        cases.append((f"n{m}", x, True))
    return cases


@pytest.mark.parametrize("case", range(len(_fold_cases())))
def test_centroid_fold_bit_exact(ctx, case):
    from pointcloudprocess_amd import ops
    name, xyz, dense = _fold_cases()[case]
    c = ora.make_cloud(xyz)
    g, cnt = ops.centroid(ctx, ops.cloud_to_device(c, ctx.device), is_dense=dense)
    e = ora.centroid(c, is_dense=dense)
    assert g[3] == 0.0
    assert _same_bytes(g[:3], e[:3]), (name, g[:3], e[:3])
    assert cnt == (len(c) if dense else int(np.isfinite(xyz).all(axis=1).sum()))


@pytest.mark.parametrize("dense", [True, False])
def test_centroid(ctx, dense):
    from pointcloudprocess_amd import ops
    c = _rand_cloud(300_000, 3, offset=(1000.0, -2000.0, 5.0), nan_every=0 if dense else 53)
    g, cnt = ops.centroid(ctx, ops.cloud_to_device(c, ctx.device), is_dense=dense)
    e = ora.centroid(c, is_dense=dense)
    assert g[3] == 0.0
    assert _same_bytes(g, e)  # the sequential fold, bit for bit
    if not dense:
        assert cnt == np.isfinite(c["x"]).sum()


@pytest.mark.parametrize("dense", [True, False])
def test_centroid_concat(ctx, dense):
    """get_rot_icp's joint centroid: ONE fold over src ++ temp (point_cloud_helper.cpp:78-83)."""
    from pointcloudprocess_amd import ops
    a = _rand_cloud(123_457, 8, offset=(3512.25, -1801.5, 40.0), nan_every=0 if dense else 61)
    b = _rand_cloud(98_765, 9, offset=(3500.0, -1790.0, 41.0), nan_every=0 if dense else 67)
    g, cnt = ops.centroid_concat(ctx, ops.cloud_to_device(a, ctx.device), ops.cloud_to_device(b, ctx.device),
                                 is_dense=dense)
    e = ora.centroid_concat(a, b, is_dense=dense)
    assert _same_bytes(g, e)


@pytest.mark.parametrize("dense", [True, False])
def test_transform_bit_exact(ctx, dense):
    from pointcloudprocess_amd import ops, synth
    c = _rand_cloud(200_000, 4, nan_every=0 if dense else 41)
    T = synth.rigid(12.0, -3.0, 7.0, (10.5, -3.25, 0.125))
    g = ops.cloud_to_host(ops.transform(ctx, ops.cloud_to_device(c, ctx.device), T, is_dense=dense))
    e = ora.transform(c, T, is_dense=dense)
    assert _same_bytes(g, e)


def test_kat_voxel_grid(ctx):
    from pointcloudprocess_amd import ops
    gk = json.load(open(os.path.join(GOLDEN, "kat_voxel_grid.json")))
    cloud = ora.make_cloud(np.array(gk["cloud_xyz"]))
    out, vidx = ops.voxel_filter(ctx, ops.cloud_to_device(cloud, ctx.device), tuple(gk["leaf"]),
                                 with_voxel_idx=True)
    out = ops.cloud_to_host(out)
    eo, ev = ora.voxel_filter(cloud, tuple(gk["leaf"]))
    assert len(out) == len(gk["expected"])
    assert _same_bytes(out, eo)
    assert np.array_equal(vidx.cpu().numpy().view(np.uint32), ev)


@pytest.mark.parametrize("leaf,all_data,dense", [
    (0.1, True, True), (0.1, False, True), ((0.05, 0.2, 0.5), True, True), (0.3, True, False),
    (1e-3, True, True),            # many singleton voxels; linear index wraps int32
])
def test_voxel_bit_exact(ctx, leaf, all_data, dense):
    from pointcloudprocess_amd import ops
    c = _rand_cloud(200_000, 5, half=20.0, offset=(3.0, -40.0, 0.0), nan_every=0 if dense else 29)
    rng = np.random.default_rng(6)
    dup = c[rng.integers(0, len(c), 20_000)]          # exact duplicates (C1: +5%)
    c = np.concatenate([c, dup])
    out, vidx = ops.voxel_filter(ctx, ops.cloud_to_device(c, ctx.device), leaf, is_dense=dense,
                                 downsample_all=all_data, with_voxel_idx=True)
    out = ops.cloud_to_host(out)
    eo, ev = ora.voxel_filter(c, leaf, is_dense=dense, downsample_all=all_data)
    assert len(out) == len(eo)
    assert np.array_equal(vidx.cpu().numpy().view(np.uint32), ev)
    assert _same_bytes(out, eo)


def test_voxel_empty(ctx):
    from pointcloudprocess_amd import ops
    out = ops.voxel_filter(ctx, torch.empty((0, 48), dtype=torch.uint8, device=ctx.device), 0.1)
    assert out.shape[0] == 0


@pytest.mark.parametrize("dense", [True, False])
def test_remove_duplicate(ctx, dense):
    """Every byte equal to the oracle's remove_duplicate with the reference's SEQUENTIAL
    centroid (point_cloud_helper.cpp:42-63), unconditionally."""
    from pointcloudprocess_amd import ops
    c = _rand_cloud(150_000, 7, half=15.0, offset=(500.0, 200.0, 10.0), nan_every=0 if dense else 31)
    g = ops.cloud_to_host(ops.remove_duplicate(ctx, ops.cloud_to_device(c, ctx.device), 0.04, is_dense=dense))
    e = ora.remove_duplicate(c, 0.04, is_dense=dense)
    assert len(g) == len(e) and _same_bytes(g, e)


def _near_face_cloud(n, leaf, seed):
    """Cloud whose points sit within ~1e-12 m of voxel faces of the centred grid: each round
    moves a subset onto c + k*leaf + tiny for the current sequential centroid c; the centroid
    moves by 1/50 of their shift, so after a few rounds they are within 1e-12 of a face."""
    rng = np.random.default_rng(seed)
    xyz = rng.uniform(-20, 20, (n, 3)) + np.array([1234.5, -987.25, 12.0])
    sel = rng.choice(n, n // 50, replace=False)
    k = rng.integers(-400, 400, (len(sel), 3))
    lf = float(np.float32(leaf))
    delta = rng.choice([-3e-13, 3e-13], (len(sel), 3))
    for _ in range(20):  # the moved points follow c, so c converges (x1/50 per round)
        c = ora.centroid(ora.make_cloud(xyz))[:3]
        xyz[sel] = (c + k * lf) + delta
    return ora.make_cloud(xyz)


def test_remove_duplicate_near_faces(ctx):
    from pointcloudprocess_amd import ops
    leaf = 0.04
    c = _near_face_cloud(200_000, leaf, 17)
    cen = ora.centroid(c)[:3]
    lf = float(np.float32(leaf))
    u = (np.stack([c["x"], c["y"], c["z"]], 1) - cen) / lf
    assert (np.abs(u - np.round(u)) < 1e-9).sum() > 1000  # many points on faces
    g = ops.cloud_to_host(ops.remove_duplicate(ctx, ops.cloud_to_device(c, ctx.device), leaf))
    e = ora.remove_duplicate(c, leaf)
    assert len(g) == len(e) and _same_bytes(g, e)


def test_remove_duplicate_c3_scale(ctx):
    """10M-point C3-like street scene, leaf 0.05: bit-exact end to end."""
    from pointcloudprocess_amd import ops, synth
    xyz = synth.street_scene(10_000_000, 3001, device="cpu").double().numpy() + np.array([500_000.0, 4_000_000.0, 30.0])
    c = ora.make_cloud(xyz)
    g = ops.cloud_to_host(ops.remove_duplicate(ctx, ops.cloud_to_device(c, ctx.device), 0.05))
    e = ora.remove_duplicate(c, 0.05)
    assert len(g) == len(e) and _same_bytes(g, e)


def test_get_rot_icp(ctx):
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid(0.3, 0.1, -0.1, (0.08, -0.05, 0.03))
    tgt, q = synth.icp_pair(60_000, 60_000, 71, 72, T_true, extent=(40.0, 40.0))
    off = np.array([3512.25, -1801.5, 40.0])
    src = ora.make_cloud(tgt.double().numpy() + off)
    tmp = ora.make_cloud(q.double().numpy() + off)
    err, M = ops.get_rot_icp(ctx, ops.cloud_to_device(src, ctx.device), ops.cloud_to_device(tmp, ctx.device),
                             0.25, iters=15)
    eerr, eM = ora.get_rot_icp(src, tmp, 0.25, 15)
    assert err > 0 and eerr > 0
    assert abs(err - eerr) <= 1e-5
    assert np.abs(M - eM).max() <= 1e-5 * max(1.0, np.abs(off).max())


def test_get_rot_icp_non_dense(ctx):
    """NaN points in either cloud: cloud_all is non-dense, the joint centroid skips them
    (point_cloud.h operator+=, point_cloud_helper.h:213-224) and ICP still registers."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid(0.3, 0.1, -0.1, (0.08, -0.05, 0.03))
    tgt, q = synth.icp_pair(60_000, 60_000, 73, 74, T_true, extent=(40.0, 40.0))
    off = np.array([3512.25, -1801.5, 40.0])
    s_xyz, t_xyz = tgt.double().numpy() + off, q.double().numpy() + off
    s_xyz[::101] = np.nan
    t_xyz[3::89, 1] = np.inf
    src, tmp = ora.make_cloud(s_xyz), ora.make_cloud(t_xyz)
    err, M = ops.get_rot_icp(ctx, ops.cloud_to_device(src, ctx.device), ops.cloud_to_device(tmp, ctx.device),
                             0.25, iters=15, src_dense=False, temp_dense=False)
    eerr, eM = ora.get_rot_icp(src, tmp, 0.25, 15, src_dense=False, tmp_dense=False)
    assert np.isfinite(M).all() and err > 0 and eerr > 0
    assert abs(err - eerr) <= 1e-5
    assert np.abs(M - eM).max() <= 1e-5 * max(1.0, np.abs(off).max())


@pytest.mark.parametrize("rmax", [0.0, -1.0])
def test_get_rot_icp_rejects_automatic_maxdist(ctx, rmax):
    """The reference's maxdist = 0 lets trimesh2 choose its threshold (point_cloud_helper.cpp:127,
    ICP.h:17-28; library absent): this build rejects it loudly instead of substituting one."""
    from pointcloudprocess_amd import _lib, ops
    src = ora.make_cloud(np.random.default_rng(5).uniform(0, 5, (2000, 3)))
    d = ops.cloud_to_device(src, ctx.device)
    with pytest.raises(_lib.PcpError) as ei:
        ops.get_rot_icp(ctx, d, d, rmax, iters=5)
    assert ei.value.code == -5  # PCP_ERR_UNSUPPORTED
