"""GPU parity of the ICP correspondence/transform loop (MI355X).

Contract (oracle/pcp_oracle.h): per query q' = R q + t (fp32 fmaf chain),
exact 1-NN within rmax by fp32 d2 = fmaf(dz,dz,fmaf(dy,dy,dx*dx)), ties by target index.
Correspondence indices and d2 are compared BIT-EXACT with the oracle at the same pose;
accumulators to 1e-7 relative (fp32 centred partial sums); full ICP poses to 1e-5
(north_star tolerance).  ICP itself is "parity unpinned" against the reference
(trimesh2 ICP() is absent).
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


def _pair(n, seed, T, extent=(40.0, 40.0)):
    from pointcloudprocess_amd import synth
    tgt, q = synth.icp_pair(n, n, seed, seed + 1, T, extent=extent)
    return tgt, q


@pytest.mark.parametrize("cell", [0.05, 0.1, 0.3])
def test_correspondence_bit_exact(ctx, cell):
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(200_000, 11, T_true)
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=cell)
    icp = ops.ICP(index, q.to(ctx.device))
    oi = ora.F32Index(tgt.numpy())
    for T in (np.eye(4), T_true, synth.rigid(0.2, 0.1, 0.1, (0.1, 0.1, -0.05))):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R = T[:3, :3].astype(np.float32)
        t = T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        gi = ci.cpu().numpy()
        gd = cd.cpu().numpy()
        assert np.array_equal(gi, ei), f"{(gi != ei).sum()} mismatching correspondences"
        assert np.array_equal(gd[ei >= 0], ed[ei >= 0])
        eacc = ora.icp_accumulate(tgt.numpy(), q.numpy(), R, t, ei, ed)
        gacc = acc.cpu().numpy()
        assert gacc[0] == eacc[0]
        # GPU: per-chunk fp32 sums of coordinates/products centred on the chunk's first
        # query, un-centred in fp64; oracle: sequential fp64.  The fp32 centred sums carry
        # ~64 * extent * 6e-8 absolute error per chunk, times the centre (|c| ~ scene size)
        # on un-centring: <= 1e-8 of the largest accumulator (measured <= 2e-9), i.e. ~1e-8
        # rad on the solved rotation, far inside the 1e-5 pose tolerance.  [23] is the
        # fallback count (diagnostic).
        scale = np.abs(eacc[:23]).max()
        assert np.allclose(gacc[:23], eacc[:23], rtol=1e-7, atol=1e-8 * scale)


@pytest.mark.parametrize("create", ["separate", "combined", "combined_auto_cell"])
def test_registration_exact_every_iteration(ctx, create):
    """A registration through both create paths (pcp_index_build_f32 + pcp_icp_create, and
    pcp_icp_create_with_target, whose query sort runs on a second stream during the target's cell
    sort -- with a given cell size, and with the automatic one, whose query sort starts only after
    the cell-size refinement): correspondences bit-exact and accumulators equal to the oracle's
    direct sums at every iteration."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(250_000, 41, T_true)
    if create == "separate":
        index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
        icp = ops.ICP(index, q.to(ctx.device))
    else:
        icp = ops.ICP.with_target(ctx, tgt.to(ctx.device), q.to(ctx.device), 0.1 if create == "combined" else 0.0)
        index = icp.index
        if create == "combined_auto_cell":
            assert 0.01 < index.cell_size < 1.0
    oi = ora.F32Index(tgt.numpy())
    T = np.eye(4)
    for it in range(10):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        gi = ci.cpu().numpy()
        assert np.array_equal(gi, ei), f"iter {it}: {(gi != ei).sum()} mismatching correspondences"
        assert np.array_equal(cd.cpu().numpy()[ei >= 0], ed[ei >= 0])
        gacc = acc.cpu().numpy().copy()
        eacc = ora.icp_accumulate(tgt.numpy(), q.numpy(), R, t, ei, ed)
        assert gacc[0] == eacc[0]
        scale = np.abs(eacc[:23]).max()
        assert np.allclose(gacc[:23], eacc[:23], rtol=1e-7, atol=1e-8 * scale), f"iter {it}"
        rc, dT = ops.icp_solve(gacc)
        assert rc == 0
        T = dT @ T
    icp.close()
    index.close()


def test_sparse_queries_over_many_bricks(ctx):
    """Few queries spread over a large target (query bricks far above ceil(nq / 256)), through
    the combined create."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, _ = _pair(400_000, 43, T_true)
    q = synth.apply_inverse(synth.street_scene(5_000, 44, extent=(50.0, 50.0)), T_true)
    icp = ops.ICP.with_target(ctx, tgt.to(ctx.device), q.to(ctx.device), 0.1)
    index = icp.index
    oi = ora.F32Index(tgt.numpy())
    for T in (np.eye(4), T_true):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        assert np.array_equal(ci.cpu().numpy(), ei)
        eacc = ora.icp_accumulate(tgt.numpy(), q.numpy(), R, t, ei, ed)
        gacc = acc.cpu().numpy()
        assert gacc[0] == eacc[0]
        assert np.allclose(gacc[:23], eacc[:23], rtol=1e-7, atol=1e-8 * np.abs(eacc[:23]).max())
    icp.close()
    index.close()


@pytest.mark.parametrize("cell,per_cell", [(0.5, 40.0), (0.5, 1500.0)])
def test_dense_cells(ctx, cell, per_cell):
    """Crowded cells: octant lists over 256 (the compare-swap top 3) and (1500 per cell) lists far
    over it, against the oracle over two poses."""
    from pointcloudprocess_amd import ops
    rng = np.random.default_rng(7)
    side = 4.0 if per_cell > 100 else 10.0
    n = int(per_cell * (side / cell) ** 3)
    tgt = rng.uniform(0, side, (n, 3)).astype(np.float32)
    q = rng.uniform(-0.2, side + 0.2, (min(n, 150_000), 3)).astype(np.float32)
    index = ops.GridIndex(ctx, torch.from_numpy(tgt).to(ctx.device), cell_size=cell)
    icp = ops.ICP(index, torch.from_numpy(q).to(ctx.device))
    oi = ora.F32Index(tgt)
    for T in (np.eye(4), _small_motion()):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q, R, t, 0.25)
        assert np.array_equal(ci.cpu().numpy(), ei)
        assert np.array_equal(cd.cpu().numpy()[ei >= 0], ed[ei >= 0])
        eacc = ora.icp_accumulate(tgt, q, R, t, ei, ed)
        gacc = acc.cpu().numpy()
        assert gacc[0] == eacc[0]
        assert np.allclose(gacc[:23], eacc[:23], rtol=1e-7, atol=1e-8 * np.abs(eacc[:23]).max())
    icp.close()
    index.close()


def _small_motion():
    from pointcloudprocess_amd import synth
    return synth.rigid(0.2, -0.1, 0.1, (0.03, -0.02, 0.01))


@pytest.mark.parametrize("cache", ["narrow", "wide"])
def test_verify_pass_exact_over_registration(ctx, cache):
    # The verify pass settles a query from its previous winner and lower bound (triangle
    # inequality); it must return exactly what an exhaustive search returns, at every
    # iteration of a registration, on a repeated pose, and after a jump back to the start.
    # Both cache record forms: 12 bytes (26-bit positions, the bound as a 12-bit code rounded
    # down; the default below 2^26 - 2 targets) and 16 bytes (PCP_ICP_OPT_WIDE_CACHE).
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(200_000, 31, T_true)
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    if cache == "wide":
        icp.set_options(wide_cache=True)
    oi = ora.F32Index(tgt.numpy())
    T = np.eye(4)
    searched = []
    poses = []
    for it in range(12):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        gi = ci.cpu().numpy()
        assert np.array_equal(gi, ei), f"iter {it}: {(gi != ei).sum()} mismatching correspondences"
        assert np.array_equal(cd.cpu().numpy()[ei >= 0], ed[ei >= 0])
        # the incremental raw-frame accounting: every accounted pair is this pose's exact winner
        # (the pair count is exact) and the accumulators match the oracle's direct sums
        gacc = acc.cpu().numpy().copy()
        eacc = ora.icp_accumulate(tgt.numpy(), q.numpy(), R, t, ei, ed)
        assert gacc[0] == eacc[0], f"iter {it}: {gacc[0]} accounted pairs, oracle {eacc[0]}"
        scale = np.abs(eacc[:23]).max()
        assert np.allclose(gacc[:22], eacc[:22], rtol=1e-7, atol=1e-8 * scale), f"iter {it}"
        assert abs(gacc[22] - eacc[22]) <= 1e-6 * eacc[22], f"iter {it}: sum d2 {gacc[22]} vs {eacc[22]}"
        searched.append(icp.last_searched())
        poses.append(T)
        rc, dT = ops.icp_solve(acc.cpu().numpy())
        assert rc == 0
        T = dT @ T
    assert searched[0] == q.shape[0]            # nothing to verify at the first launch
    assert searched[-1] < 0.75 * q.shape[0], searched  # settled ones skip the search
    # the same pose again: every settled query verifies (zero motion)
    _, ci, _ = icp.step(poses[-1], 0.25, corr=True)
    R, t = poses[-1][:3, :3].astype(np.float32), poses[-1][:3, 3].astype(np.float32)
    ei, _ = oi.correspond(q.numpy(), R, t, 0.25)
    assert np.array_equal(ci.cpu().numpy(), ei)
    # a jump back to the identity: the bounds no longer hold for most queries
    _, ci, _ = icp.step(np.eye(4), 0.25, corr=True)
    ei, _ = oi.correspond(q.numpy(), np.eye(3, dtype=np.float32), np.zeros(3, np.float32), 0.25)
    assert np.array_equal(ci.cpu().numpy(), ei)
    # a smaller rmax than the bounds were made with
    _, ci, _ = icp.step(poses[-1], 0.02, corr=True)
    ei, _ = oi.correspond(q.numpy(), R, t, 0.02)
    assert np.array_equal(ci.cpu().numpy(), ei)


@pytest.mark.parametrize("cache", ["narrow", "wide"])
def test_long_registration_history_wrap(ctx, cache):
    """75 launches of small motions: the caches outlive the pose history (64 slots narrow, 256
    wide) and age out (32 / 128 launches) -- correspondences stay exact at every checked launch."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(100_000, 53, T_true)
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    if cache == "wide":
        icp.set_options(wide_cache=True)
    oi = ora.F32Index(tgt.numpy())
    rng = np.random.default_rng(5)
    for it in range(75):
        T = synth.rigid(*(rng.normal(0, 0.05, 3)), tuple(rng.normal(0, 0.004, 3))) @ T_true
        _, ci, cd = icp.step(T, 0.25, corr=True)
        if it % 5 == 4 or it >= 70:
            R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
            ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
            assert np.array_equal(ci.cpu().numpy(), ei), f"launch {it}"
            assert np.array_equal(cd.cpu().numpy()[ei >= 0], ed[ei >= 0])
    icp.close()
    index.close()


def test_ties_lattice(ctx):
    from pointcloudprocess_amd import ops
    # integer lattice target + half-integer queries: every query has 8 equidistant targets
    g = np.stack(np.meshgrid(np.arange(20), np.arange(20), np.arange(5), indexing="ij"), -1)
    tgt = g.reshape(-1, 3).astype(np.float32)
    q = (tgt[:500] + 0.5).astype(np.float32)
    index = ops.GridIndex(ctx, torch.from_numpy(tgt).to(ctx.device), cell_size=1.0)
    icp = ops.ICP(index, torch.from_numpy(q).to(ctx.device))
    ei, ed = ora.F32Index(tgt).correspond(q, np.eye(3), np.zeros(3), 1.0)
    for _ in range(2):  # the second launch starts from the first one's winners and bounds
        _, ci, cd = icp.step(np.eye(4), 1.0, corr=True)
        assert np.array_equal(ci.cpu().numpy(), ei)


def test_far_queries_rejected_and_failure(ctx):
    from pointcloudprocess_amd import ops
    tgt = torch.rand((1000, 3)) * 10
    q = torch.rand((100, 3)) * 10 + 1000.0  # nowhere near the target
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.5)
    icp = ops.ICP(index, q.to(ctx.device))
    acc, ci, cd = icp.step(np.eye(4), 0.5, corr=True)
    assert (ci.cpu().numpy() == -1).all()
    assert acc.cpu().numpy()[0] == 0
    err, T = icp.run(np.eye(4), 0.5, 5)
    assert err < 0  # ICP.h:26-28: failure => err < 0


def test_empty_query(ctx):
    from pointcloudprocess_amd import ops
    tgt = torch.rand((1000, 3))
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, torch.zeros((0, 3)).to(ctx.device))
    acc = icp.step(np.eye(4), 0.5)
    assert acc.cpu().numpy()[0] == 0


def test_icp_run_matches_oracle(ctx):
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(300_000, 21, T_true)
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    err, T = icp.run(np.eye(4), 0.25, 20)
    eerr, eT = ora.icp(tgt.numpy(), q.numpy(), np.eye(4), 0.25, 20)
    assert err > 0 and abs(err - eerr) < 1e-5
    assert np.abs(T - eT).max() < 1e-5


def test_device_loop_matches_oracle_and_host_loop(ctx):
    # pcp_icp_run_dev / step_dev + solve_dev: pose, solve and stats stay in device memory
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(300_000, 21, T_true)
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    T_dev, stats = icp.new_pose()
    icp.run_dev(T_dev, stats, 0.25, 20)
    ms, nl = icp.kernel_ms()
    assert nl == 20 and ms > 0
    st = stats.cpu().numpy()
    assert st[0] == 0 and st[3] == 20
    T = T_dev.cpu().numpy().reshape(4, 4)
    eerr, eT = ora.icp(tgt.numpy(), q.numpy(), np.eye(4), 0.25, 20)
    assert abs(st[1] - eerr) < 1e-5
    assert np.abs(T - eT).max() < 1e-5
    # the same iterations through step_dev + solve_dev equal run_dev exactly on a fresh engine
    # (the accumulators' summation order follows which pass -- verify, search or fallback --
    # settled each query, and that depends on the engine's carried winners and bounds)
    icp2 = ops.ICP(index, q.to(ctx.device))
    T2, st2 = icp2.new_pose()
    for _ in range(20):
        icp2.solve_dev(icp2.step_dev(T2, 0.25), T2, st2)
    assert torch.equal(T2, T_dev) and torch.equal(st2, stats)
    icp2.close()
    # a warm engine (carried state) gives the same correspondences: poses equal to rounding
    T3, st3 = icp.new_pose()
    icp.run_dev(T3, st3, 0.25, 20)
    assert (T3 - T_dev).abs().max().item() < 1e-7 and st3[3].item() == 20
    # and the host loop (host solve): same arithmetic, but a last-bit difference of the fp64
    # solve can flip the fp32 cast of the pose and with it a few correspondences
    herr, hT = icp.run(np.eye(4), 0.25, 20)
    assert np.abs(hT - T).max() < 1e-6 and abs(herr - st[1]) < 1e-6


def test_device_loop_graph_replay_equals_plain_launches(ctx):
    """With PCP_ICP_OPT_GRAPH, device-pose launches after the first replay one captured HIP graph of
    the verify .. fallback section (the launch index is read from the device).  Its accumulators equal, bit for bit, those
    of plain launches at the same poses on a second engine (the host-pose path with correspondence
    output never uses the graph), and those plain launches' correspondences equal the oracle's."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(200_000, 61, T_true)
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    icp.set_options(graph=True)
    T_dev, stats = icp.new_pose()
    poses, accs = [], []
    for _ in range(12):
        poses.append(T_dev.cpu().numpy().reshape(4, 4).copy())
        acc = icp.step_dev(T_dev, 0.25)
        accs.append(acc.cpu().numpy().copy())
        icp.solve_dev(acc, T_dev, stats)
    icp2 = ops.ICP(index, q.to(ctx.device))
    oi = ora.F32Index(tgt.numpy())
    for it, T in enumerate(poses):
        acc2, ci, _ = icp2.step(T, 0.25, corr=True)
        assert np.array_equal(acc2.cpu().numpy(), accs[it]), f"iteration {it}"
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, _ = oi.correspond(q.numpy(), R, t, 0.25)
        assert np.array_equal(ci.cpu().numpy(), ei), f"iteration {it}"
    icp2.close()
    icp.close()
    index.close()


def test_device_loop_failure_latches(ctx):
    from pointcloudprocess_amd import ops
    tgt = torch.rand((1000, 3)) * 10
    q = torch.rand((100, 3)) * 10 + 1000.0  # no correspondences: the solve fails
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.5)
    icp = ops.ICP(index, q.to(ctx.device))
    T_dev, stats = icp.new_pose()
    icp.run_dev(T_dev, stats, 0.5, 3)
    st = stats.cpu().numpy()
    assert st[0] == -1 and st[3] == 0
    assert np.array_equal(T_dev.cpu().numpy().reshape(4, 4), np.eye(4))


def test_sparse_grid_matches_oracle(ctx):
    # two clusters 5 km apart with 5 cm cells: the dense cell table would exceed its budget,
    # so the index uses 4x4x4 bricks and the ICP runs the general box search for every query
    from pointcloudprocess_amd import ops, synth
    rng = np.random.default_rng(4)
    a = rng.uniform(0, 2, size=(20000, 3)).astype(np.float32)
    tgt = np.concatenate([a, a[:5000] + np.float32(5000.0)])
    q = (tgt + rng.normal(scale=0.01, size=tgt.shape)).astype(np.float32)
    index = ops.GridIndex(ctx, torch.from_numpy(tgt).to(ctx.device), cell_size=0.05)
    assert ctx.lib.pcp_index_cells(index.h) < 1e9  # sparse (brick) mode
    icp = ops.ICP(index, torch.from_numpy(q).to(ctx.device))
    T = synth.rigid(0.1, 0.0, 0.0, (0.01, 0.0, 0.0))
    acc, ci, cd = icp.step(T, 0.1, corr=True)
    ei, ed = ora.F32Index(tgt).correspond(q, T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32), 0.1)
    assert np.array_equal(ci.cpu().numpy(), ei)


def test_target_sharded_keys_match_oracle(ctx):
    """Target-sharded mode emulated on one GPU: two shard engines, MIN of
    their keys = the oracle's global correspondences (bit-exact); the per-shard accumulators
    sum to the oracle's fp64 accumulators (same exact products, different order)."""
    import torch
    from pointcloudprocess_amd import distributed as D, synth
    T_true = synth.rigid()
    tgt, q = _pair(120_000, 31, T_true)
    n = tgt.shape[0]
    dq = q.to(ctx.device)
    shards = [D.shard_range(n, 2, r) for r in range(2)]
    engines = [D.GpuEngine(ctx, tgt[lo:hi].to(ctx.device), dq, cell_size=0.1) for lo, hi in shards]
    T = synth.rigid(0.1, 0.05, 0.0, (0.02, 0.01, 0.0))
    keys = torch.minimum(engines[0].keys(T, 0.25, shards[0][0]), engines[1].keys(T, 0.25, shards[1][0]))
    k = keys.cpu().numpy()
    R = T[:3, :3].astype(np.float32)
    t = T[:3, 3].astype(np.float32)
    ei, ed = ora.F32Index(tgt.numpy()).correspond(q.numpy(), R, t, 0.25)
    none = k == np.iinfo(np.int64).max
    assert np.array_equal(none, ei < 0)
    assert np.array_equal((k[~none] & 0xFFFFFFFF).astype(np.int32), ei[~none])
    assert np.array_equal((k[~none] >> 32).astype(np.uint32).view(np.float32), ed[~none])
    acc = sum(e.accumulate_keys(T, keys, lo, hi).cpu().numpy().copy() for e, (lo, hi) in zip(engines, shards))
    eacc = ora.icp_accumulate(tgt.numpy(), q.numpy(), R, t, ei, ed)
    assert np.allclose(acc[:23], eacc[:23], rtol=1e-12, atol=1e-12 * np.abs(eacc[:23]).max())
    for e in engines:
        e.close()


def test_target_sharded_dev_owned_form(ctx):
    """Device-resident target-sharded loop pieces (keys_dev + keys_owner + accumulate_owned), two
    shard engines on one GPU, each holding ONLY its x-slab of the target: most queries lie
    outside a shard's grid (the octant pass's out-of-grid exit, then the verify passes).  The
    MIN of the keys = the oracle's global correspondences bit-exact at every pose of a
    sequence; the owners of the winners split the queries, and the two ranks' accumulators --
    each over the queries whose winner it owns, read from its own shard -- sum to the
    oracle's."""
    import torch
    from pointcloudprocess_amd import distributed as D, ops, synth
    tgt, q = _pair(150_000, 33, synth.rigid())
    tgt = tgt[torch.argsort(tgt[:, 0])].contiguous()  # global index = x order: slabs
    n, nq = tgt.shape[0], q.shape[0]
    dq = q.to(ctx.device)
    bounds = [D.shard_range(n, 2, r)[0] for r in range(2)] + [n]
    engines = [D.GpuEngine(ctx, tgt[bounds[r]:bounds[r + 1]].to(ctx.device), dq, cell_size=0.1) for r in range(2)]
    bnd = torch.tensor(bounds, dtype=torch.int64, device=ctx.device)
    T_dev, _ = engines[0].new_pose(np.eye(4))
    ix = ora.F32Index(tgt.numpy())
    for T in (np.eye(4), synth.rigid(0.1, 0.05, 0.0, (0.02, 0.01, 0.0)), synth.rigid(0.3, 0.1, -0.05, (0.1, 0.0, 0.02)),
              synth.rigid(0.1, 0.05, 0.0, (0.02, 0.01, 0.0))):
        T_dev.copy_(torch.from_numpy(np.ascontiguousarray(T.reshape(16))).to(ctx.device))
        local = [engines[r].keys_dev(T_dev, 0.25, bounds[r]).clone() for r in range(2)]
        keys = torch.minimum(local[0], local[1])
        k = keys.cpu().numpy()
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = ix.correspond(q.numpy(), R, t, 0.25)
        none = k == np.iinfo(np.int64).max
        assert np.array_equal(none, ei < 0)
        assert np.array_equal((k[~none] & 0xFFFFFFFF).astype(np.int32), ei[~none])
        assert np.array_equal((k[~none] >> 32).astype(np.uint32).view(np.float32), ed[~none])
        owner = ops.keys_owner(ctx, keys, bnd)
        o = owner.cpu().numpy()
        assert np.array_equal(o == 255, none)
        assert np.array_equal(o[~none], (ei[~none] >= bounds[1]).astype(np.uint8))
        acc = sum(engines[r].accumulate_owned(T_dev, local[r], owner, r, bounds[r], bounds[r + 1]).cpu().numpy().copy()
                  for r in range(2))
        eacc = ora.icp_accumulate(tgt.numpy(), q.numpy(), R, t, ei, ed)
        assert np.allclose(acc[:23], eacc[:23], rtol=1e-12, atol=1e-12 * np.abs(eacc[:23]).max())
    for e in engines:
        e.close()


def test_slab_guard_device(ctx):
    from pointcloudprocess_amd import ops
    flag = torch.zeros(1, dtype=torch.int32, device=ctx.device)
    T = np.eye(4)
    box = [0.0, 10.0, -5.0, 5.0, 0.0, 2.0]
    ops.slab_guard(ctx, torch.from_numpy(T.reshape(16).copy()).to(ctx.device), box, -1.0, 11.0, flag)
    assert flag.item() == 0
    T[0, 3] = 1.5
    ops.slab_guard(ctx, torch.from_numpy(T.reshape(16).copy()).to(ctx.device), box, -1.0, 11.0, flag)
    assert flag.item() == 1


@pytest.mark.parametrize("gs", ["2,2", "4,4", "8,8", "1,0"])
def test_octant_lane_groups_exact(ctx, gs):
    """G lanes per query in the octant pass (pcp_icp_set_options "first,list"; 0 = by density):
    the group merge, the per-group cache write and the > 256-candidate compare-swap path must
    give the oracle's correspondences over a registration, on lattice ties and a dense cluster."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(120_000, 51, T_true)
    rng = np.random.default_rng(52)
    c0 = tgt[0].numpy()
    cluster = (c0 + rng.uniform(-0.02, 0.02, (3000, 3))).astype(np.float32)  # >256 points per cell
    lat = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    lat = (lat * 0.1 + np.array([5.0, 5.0, 20.0])).astype(np.float32)       # exact ties
    tgt = torch.from_numpy(np.concatenate([tgt.numpy(), cluster, lat]))
    qn = np.concatenate([q.numpy(), cluster[:500] + 0.003, (lat + 0.05).astype(np.float32)])
    q = torch.from_numpy(qn.astype(np.float32))
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    first, lst = (int(v) for v in gs.split(","))
    icp.set_options(oct_lanes_first=first, oct_lanes_list=lst)
    oi = ora.F32Index(tgt.numpy())
    T = np.eye(4)
    for it in range(6):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        gi = ci.cpu().numpy()
        assert np.array_equal(gi, ei), f"G {gs} iter {it}: {(gi != ei).sum()} mismatching correspondences"
        assert np.array_equal(cd.cpu().numpy()[ei >= 0], ed[ei >= 0])
        rc, dT = ops.icp_solve(acc.cpu().numpy())
        assert rc == 0
        T = dT @ T


@pytest.mark.parametrize("lanes", ["1", "2", "4", "8"])
def test_fallback_lane_groups_exact(ctx, lanes):
    """G lanes per query in the fallback pass (pcp_icp_set_options; the default picks G from the
    list length): the strided row scans, the per-plane group merge and box_search's group-bound
    row cuts must give the oracle's correspondences.  Cells of rmax / 2.5 over a sparse scan send many
    queries through box_search, including "nothing within rmax" boxes; lattice ties and a dense
    cluster exercise the (d2, index) order."""
    from pointcloudprocess_amd import ops, synth
    T_true = synth.rigid()
    tgt, q = _pair(60_000, 61, T_true, extent=(30.0, 30.0))  # a dense cell table
    rng = np.random.default_rng(62)
    c0 = tgt[0].numpy()
    cluster = (c0 + rng.uniform(-0.02, 0.02, (800, 3))).astype(np.float32)
    lat = np.stack(np.meshgrid(np.arange(6), np.arange(6), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    lat = (lat * 0.1 + np.array([5.0, 5.0, 1.0])).astype(np.float32)
    tgt = torch.from_numpy(np.concatenate([tgt.numpy(), cluster, lat]))
    qn = np.concatenate([q.numpy(), cluster[:200] + 0.003, (lat + 0.05).astype(np.float32),
                         (lat + np.array([0.0, 0.0, 0.2], np.float32)).astype(np.float32)])
    q = torch.from_numpy(qn.astype(np.float32))
    index = ops.GridIndex(ctx, tgt.to(ctx.device), cell_size=0.1)
    icp = ops.ICP(index, q.to(ctx.device))
    icp.set_options(ring_lanes=int(lanes))
    oi = ora.F32Index(tgt.numpy())
    T = np.eye(4)
    fallbacks = 0
    for it in range(5):
        acc, ci, cd = icp.step(T, 0.25, corr=True)
        fallbacks += icp.last_fallback()
        R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
        ei, ed = oi.correspond(q.numpy(), R, t, 0.25)
        gi = ci.cpu().numpy()
        assert np.array_equal(gi, ei), f"G {lanes} iter {it}: {(gi != ei).sum()} mismatching correspondences"
        assert np.array_equal(cd.cpu().numpy()[ei >= 0], ed[ei >= 0])
        rc, dT = ops.icp_solve(acc.cpu().numpy())
        assert rc == 0
        T = dT @ T
    assert fallbacks > 200  # the fallback pass really ran on a list
