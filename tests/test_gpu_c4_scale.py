"""Bench-scale C4 parity (BASELINE.json configs[3], the bench's own workload): 50M-vs-50M
street scene, grid cell 0.12 m (bench.py's), rmax 0.25.  The registration runs through the
same candidate-cache engine the bench times; at iterations 0, 1, 5 and 19 a seeded random
sample of 1M queries is compared BIT-EXACT with the oracle's exhaustive kd-tree
correspondences (index and fp32 d2), and the accumulators over all 50M queries agree with
the oracle's to 1e-7 relative.  Also: do_scale through the device solve (k_icp_solve_dev,
main_blend.cpp:818 get_rot_icp(..., true, false)) against the oracle solve.
ICP itself is "parity unpinned" (trimesh2 is absent); the contract is DESIGN.md §6.4."""
import numpy as np
import pytest
import torch

import oracle_ctypes as ora

pytestmark = pytest.mark.gpu

N = 50_000_000
CHECK = (0, 1, 5, 19)


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


def test_c4_bench_scale_correspondences(ctx):
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = synth.icp_pair(N, N, 4001, 4002, T_true, device=ctx.device)  # bench.py's seeds
    tgt_h, q_h = tgt.cpu().numpy(), q.cpu().numpy()
    ix = ora.F32Index(tgt_h)
    index = ops.GridIndex(ctx, tgt, cell_size=0.12)
    icp = ops.ICP(index, q)
    rng = np.random.default_rng(4003)
    sample = np.sort(rng.choice(N, 1_000_000, replace=False))
    T = np.eye(4)
    for it in range(CHECK[-1] + 1):
        check = it in CHECK
        acc, ci, cd = icp.step(T, 0.25, corr=True) if check else (icp.step(T, 0.25), None, None)
        a = acc.cpu().numpy().copy()
        if check:
            R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
            gi, gd = ci.cpu().numpy(), cd.cpu().numpy()
            ei, ed = ix.correspond(q_h[sample], R, t, 0.25)
            assert np.array_equal(gi[sample], ei), f"iteration {it}: indices differ"
            assert np.array_equal(gd[sample].view(np.uint32), ed.view(np.uint32)), f"iteration {it}: d2 differ"
            fi, fd = ix.correspond(q_h, R, t, 0.25)  # every query, for the accumulators
            eacc = ora.icp_accumulate(tgt_h, q_h, R, t, fi, fd)
            assert a[0] == eacc[0]
            scale = np.abs(eacc[:23]).max()
            assert np.allclose(a[:23], eacc[:23], rtol=1e-7, atol=1e-7 * scale), f"iteration {it}"
        rc, dT = ops.icp_solve(a)
        assert rc == 0
        T = dT @ T
    assert np.abs(T - T_true).max() < 2e-3
    icp.close()
    index.close()


def test_device_solve_do_scale(ctx):
    """k_icp_solve_dev with do_scale (Umeyama scale) against the oracle's solve."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid(0.4, 0.1, -0.2, (0.1, -0.05, 0.03))
    tgt, q = synth.icp_pair(200_000, 200_000, 91, 92, T_true, extent=(40.0, 40.0))
    q = q * 1.002  # a small scale difference for the Umeyama scale to recover
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    T_dev, stats = icp.new_pose()
    for _ in range(3):
        acc = icp.step_dev(T_dev, 0.25)
        a = acc.cpu().numpy().copy()
        T_prev = T_dev.cpu().numpy().reshape(4, 4).copy()
        icp.solve_dev(acc, T_dev, stats, do_scale=True)
        rc, dT = ora.icp_solve(a, do_scale=True)
        assert rc == 0
        got = T_dev.cpu().numpy().reshape(4, 4)
        assert np.abs(got - dT @ T_prev).max() < 1e-9
    s = np.cbrt(np.linalg.det(T_dev.cpu().numpy().reshape(4, 4)[:3, :3]))
    assert 1 / 1.002 - 1e-3 < s < 0.9995, s  # the scale is being recovered (3 iterations)
    icp.close()
    index.close()
