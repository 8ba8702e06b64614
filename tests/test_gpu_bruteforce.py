"""GPU parity of the MFMA brute-force kNN (BASELINE config C2) against the oracle.

fp32 MFMA ranking + certified fp64 re-rank: indices and d2 must be
BIT-EXACT with the oracle's nearestKSearch (FLANN L2_Simple<double>, ties by index).
"""
import numpy as np
import pytest
import torch

import oracle_ctypes as ora

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


def _dev(ctx, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(ctx.device)


@pytest.mark.parametrize("k", [1, 8, 12, 32])
def test_bruteforce_bit_exact(ctx, k):
    from pointcloudprocess_amd import ops, synth
    t = synth.uniform_cube(40_000, 2001, half=50.0).numpy()
    q = np.concatenate([synth.uniform_cube(6_000, 2002, half=55.0).numpy(), t[:1000]])
    gi, gd = ops.knn_bruteforce(ctx, _dev(ctx, t), _dev(ctx, q), k)
    ei, ed = ora.KdTree(t).knn(q, k)
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    print(f"k={k}: fallback queries {ops.knn_bruteforce_last_fallback(ctx)}")
    assert np.array_equal(gi, ei), f"{(gi != ei).any(1).sum()} rows differ"
    assert np.array_equal(gd, ed)


def test_bruteforce_ties_and_fallback(ctx):
    """Integer lattice: massive exact ties force uncertified rows through the fp64 scan."""
    from pointcloudprocess_amd import ops
    g = np.stack(np.meshgrid(np.arange(16), np.arange(16), np.arange(16), indexing="ij"), -1)
    t = g.reshape(-1, 3).astype(np.float64)
    t = t[np.random.default_rng(5).permutation(len(t))]
    q = t[:700] + 0.5
    gi, gd = ops.knn_bruteforce(ctx, _dev(ctx, t), _dev(ctx, q), 8)
    ei, ed = ora.KdTree(t).knn(q, 8)
    assert np.array_equal(gi.cpu().numpy(), ei)
    assert np.array_equal(gd.cpu().numpy(), ed)


def test_bruteforce_nonfinite_small_and_aos(ctx):
    from pointcloudprocess_amd import ops, synth
    t = synth.uniform_cube(3000, 7, half=5.0).numpy()
    t[::13] = np.nan
    q = synth.uniform_cube(500, 8, half=5.0).numpy()
    tc = ora.make_cloud(t)
    gi, gd = ops.knn_bruteforce(ctx, ops.cloud_to_device(tc, ctx.device), _dev(ctx, q), 8)
    ei, ed = ora.KdTree(t).knn(q, 8)
    assert np.array_equal(gi.cpu().numpy(), ei) and np.array_equal(gd.cpu().numpy(), ed)
    t5 = t[1:6]
    gi, gd = ops.knn_bruteforce(ctx, _dev(ctx, t5), _dev(ctx, q), 8)   # k > n: padded
    ei, ed = ora.KdTree(t5).knn(q, 8)
    assert np.array_equal(gi.cpu().numpy(), ei) and np.array_equal(gd.cpu().numpy(), ed)
