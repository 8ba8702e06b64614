"""F3 calculate_plan_parameter_rpca (calculate_feature.cpp:208-368) on the GPU (rpca.hip)
against the oracle's restatement (ora_rpca) of the same deterministic contract: every field
of every LAS_POINT_PROPERTY record identical (normals, Distance, curvature as the floats and
doubles the reference stores).  kNN(20) rows come from pcp_knn (bit-exact vs the oracle's
kd-tree, tests/test_gpu_knn.py).  Parity vs the reference itself is unpinned: it seeds rand()
with time(NULL) and takes OpenCV's eigenvector sign."""
import numpy as np
import pytest
import torch

import oracle_ctypes as ora

pytestmark = pytest.mark.gpu
FIELDS = ("normal_x", "normal_y", "normal_z", "distance", "curvature", "point_id")


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


def _bits(a):
    return np.ascontiguousarray(a).tobytes()


def _rows(ctx, xyz):
    from pointcloudprocess_amd import ops
    d = torch.from_numpy(xyz).to(ctx.device)
    index = ops.GridIndex(ctx, d)  # fp64 (KdTreeFLANN contract) for float64 clouds
    idx, _ = ops.knn(index, d, 20)
    return d, idx, index


@pytest.mark.parametrize("seed", [0, 12345])
def test_rpca_matches_oracle_street_scene(ctx, seed):
    from pointcloudprocess_amd import ops, synth
    xyz = synth.street_scene(60_000, 3101, extent=(40.0, 40.0), noise=0.01).double().numpy()
    rng = np.random.default_rng(3)
    out = rng.choice(len(xyz), 600, replace=False)  # 1 % outliers
    xyz[out] += rng.normal(0, 0.3, (len(out), 3))
    d, idx, index = _rows(ctx, xyz)
    g = ops.normals_rpca(ctx, d, idx, seed=seed).cpu().numpy().view(ops.POINT_PROPERTY).reshape(-1)
    e = ora.rpca(xyz, idx.cpu().numpy(), seed=seed)
    for f in FIELDS:
        assert _bits(g[f]) == _bits(e[f]), (f, int((g[f] != e[f]).sum()))
    assert (g["segment_id"] == 0).all()
    assert (np.abs(g["normal_z"]) > 0.99).mean() > 0.3  # the ground is a large part of the scene


def test_rpca_short_rows_and_unsupported(ctx):
    from pointcloudprocess_amd import ops
    xyz = np.random.default_rng(1).uniform(-1, 1, (500, 3))
    d, idx, index = _rows(ctx, xyz)
    idx[:7, 2:] = -1  # N <= 3: {0, 0, 0, curvature 1}
    g = ops.normals_rpca(ctx, d, idx).cpu().numpy().view(ops.POINT_PROPERTY).reshape(-1)
    e = ora.rpca(xyz, idx.cpu().numpy())
    for f in FIELDS:
        assert _bits(g[f]) == _bits(e[f]), (f, int((g[f] != e[f]).sum()))
    assert (g["curvature"][:7] == 1.0).all() and (g["normal_x"][:7] == 0).all()
    wide = torch.cat([idx, idx[:, :1]], dim=1)  # k = 21 > the reference's 20
    with pytest.raises(Exception):
        ops.normals_rpca(ctx, d, wide)
