"""GPU parity of the cloud passes (MI355X) against the oracle.

V2 getMinMax3D, I2 transformPointCloud, V3 VoxelGrid::applyFilter: BIT-EXACT (every byte
of every 48-byte output record, plus the u32 voxel index), including the reference KAT
(tests/golden/kat_voxel_grid.json, main_test.cpp:126-154) and the int32 wrap of the
linear voxel index.  I3 compute3DCentroid: the GPU sums in a fixed tree order, the
reference folds sequentially -> 1e-12 relative.  V4 remove_duplicate: bit-exact given the
same centroid (ora_remove_duplicate_c), close to the sequential-centroid oracle.
I1 get_rot_icp: pose within 1e-5 (north_star tolerance; ICP is "parity unpinned").
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


@pytest.mark.parametrize("dense", [True, False])
def test_centroid(ctx, dense):
    from pointcloudprocess_amd import ops
    c = _rand_cloud(300_000, 3, offset=(1000.0, -2000.0, 5.0), nan_every=0 if dense else 53)
    g, cnt = ops.centroid(ctx, ops.cloud_to_device(c, ctx.device), is_dense=dense)
    e = ora.centroid(c, is_dense=dense)
    assert g[3] == 0.0
    assert np.allclose(g[:3], e[:3], rtol=1e-12, atol=0)
    if not dense:
        assert cnt == np.isfinite(c["x"]).sum()


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
    from pointcloudprocess_amd import ops
    c = _rand_cloud(150_000, 7, half=15.0, offset=(500.0, 200.0, 10.0), nan_every=0 if dense else 31)
    dc = ops.cloud_to_device(c, ctx.device)
    g = ops.cloud_to_host(ops.remove_duplicate(ctx, dc, 0.04, is_dense=dense))
    gc, _ = ops.centroid(ctx, dc, is_dense=dense)
    e = ora.remove_duplicate_c(c, 0.04, gc, is_dense=dense)   # same centroid: bit-exact
    assert len(g) == len(e) and _same_bytes(g, e)
    e2 = ora.remove_duplicate(c, 0.04, is_dense=dense)        # sequential centroid
    if len(e2) == len(g):
        assert np.allclose(g["x"], e2["x"], rtol=0, atol=1e-9)


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
