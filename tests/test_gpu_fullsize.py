"""Full-size parity at the BASELINE.json configs, against the oracle (test infrastructure).

The per-kernel parity tests elsewhere run at sizes chosen for speed; these run the exact bench
workloads of bench_configs.py (same generators, seeds and device RNG streams), so a kernel change
that only misbehaves at the bench's density or size cannot pass as "bit-identical to another GPU
path":

* C2 (configs[1]): 1M-vs-1M uniform cube, k = 8 -- indices and d2 BIT-EXACT against the
  oracle's exact kd-tree (FLANN nearestKSearch contract, kd_tree.h:814-845).
* C3 (configs[2]): the 10M-point street scene (seed 3001), VoxelGrid leaf 0.05f (every byte
  of the ~8.86M centroids, voxel_grid.h:811-1056) and then calculate_feature normals k = 32 over
  the centroids (calculate_feature.cpp:119-206 over kd_tree.h:814-845 neighbourhoods), every row
  against the oracle to the same 1e-6 tolerance as test_gpu_knn.py::test_normals_vs_oracle;
  the bit-identical row fraction is printed.
* C5 (configs[4]): the bench's 200M-point scene, radius r = 0.2 over the fp16 cell-relative
  index (~12.8e9 CSR entries, past 2^31): every row is checked on the device (no entry at or past
  r + eps, its own point once); a 200K-query sample from 20 tiles against the oracle's exact fp64
  radiusSearch (kd_tree.h:863-903) built on each tile +- 1 m, with the fp16 band:
  no duplicates, as many points closer than r - eps as the oracle finds; rows with no point
  inside the band have their F1 normals compared with the oracle's fp64 plane of the (then
  identical) neighbour set, as an angle.
"""
import math

import numpy as np
import pytest
import torch

import oracle_ctypes as ora

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


def test_c2_fullsize_bit_exact(ctx):
    from pointcloudprocess_amd import ops, synth
    n = 1_000_000
    t = synth.uniform_cube(n, 2001, half=50.0, device=ctx.device)   # bench_configs.cfg_c2, rank 0
    q = synth.uniform_cube(n, 2002, half=50.0, device=ctx.device)
    gi, gd = ops.knn_bruteforce(ctx, t, q, 8)
    fb = ops.knn_bruteforce_last_fallback(ctx)
    gi, gd = gi.cpu().numpy(), gd.cpu().numpy()
    ei, ed = ora.KdTree(t.cpu().numpy()).knn(q.cpu().numpy(), 8)
    bad = (gi != ei).any(1) | (gd != ed).any(1)
    print(f"C2 1M x 1M k=8: fallback queries {fb}, differing rows {int(bad.sum())}")
    assert not bad.any()


def test_c3_fullsize_voxel_and_normals(ctx):
    import bench_configs
    from pointcloudprocess_amd import ops
    n = 10_000_000
    cloud = bench_configs.street_aos48(n, 3001, ctx.device)            # bench_configs.cfg_c3, rank 0
    vox = ops.voxel_filter(ctx, cloud, 0.05)
    host = ops.cloud_to_host(cloud)
    evox, _ = ora.voxel_filter(host, 0.05)
    gvox = ops.cloud_to_host(vox)
    print(f"C3 voxel: {n} points -> {len(gvox)} centroids (oracle {len(evox)})")
    assert len(gvox) == len(evox)
    assert np.array_equal(gvox.view(np.uint8), evox.view(np.uint8)), "voxel bytes differ"
    del host, evox

    ix = ops.GridIndex(ctx, vox, stride_bytes=48)
    g = ops.normals_knn(ix, 32).cpu().numpy()
    ix.close()
    vx = np.stack([gvox["x"], gvox["y"], gvox["z"]], 1)
    e = ora.normals_knn(vx, 32)
    ev = np.stack([e[f] for f in ("normal_x", "normal_y", "normal_z", "min_value", "curvature", "distance")], 1)
    diff = np.abs(g - ev)
    exact = (g == ev).all(1).mean()
    worst = int(np.argmax((diff / np.maximum(1.0, np.abs(ev))).max(1)))
    print(f"C3 normals k=32 over {len(vx)} centroids: bit-identical rows {exact:.6f}, max |diff| {diff.max():.3e} "
          f"(row {worst})")
    assert np.all(diff <= 1e-6 * np.maximum(1.0, np.abs(ev)))


def test_c5_fullsize_200m(ctx):
    """The C5 bench scene itself (bench_configs.cfg_c5, rank 0): 200M points, ~12.8e9 CSR entries
    (past 2^31: 64-bit offsets and row positions).  Every row: offsets monotone, each row holds its
    own point, no entry at or beyond r + eps from its query (exact fp64 distance on the fp32 input).
    A 200K-query sample from 20 tiles of 4 x 4 m is band-checked against the oracle kd-tree built on
    each tile +- 1 m, and the band-free rows' normals against the oracle's fp64 planes (as angles)."""
    from h16_check import EPS, angle_summary, check_against_oracle
    from pointcloudprocess_amd import ops, synth
    R = 0.2
    n = 200_000_000
    side = math.sqrt(n / 1.5e6) * 40.0                 # bench_configs.cfg_c5's scene
    xyz = synth.street_scene(n, 5001, extent=(side, side), device=ctx.device)
    ix = ops.H16Index(ctx, xyz, cell_size=R)
    offs, idx, nrm = ix.radius_normals(R)
    ix.close()
    nnz = idx.numel()
    lens = offs[1:] - offs[:-1]
    print(f"C5 200M: nnz {nnz} (2^31 = {2 ** 31}), nbar {nnz / n:.1f}, max row {int(lens.max())}")
    assert nnz > 2 ** 31 and int(offs[0]) == 0 and int(offs[-1]) == nnz and bool((lens >= 1).all())
    # every row, in chunks of rows: nothing at or beyond r + eps; the query itself present
    far = 0
    self_missing = 0
    chunk = 2_000_000
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        e0, e1 = int(offs[r0]), int(offs[r1])
        ent = idx[e0:e1].long()
        row_of = torch.repeat_interleave(torch.arange(r0, r1, device=ctx.device), lens[r0:r1])
        d2 = ((xyz[ent].double() - xyz[row_of].double()) ** 2).sum(1)
        far += int((d2 >= (R + EPS) ** 2).sum())
        has_self = torch.zeros(r1 - r0, dtype=torch.int32, device=ctx.device).index_add_(
            0, row_of - r0, (ent == row_of).int())
        self_missing += int((has_self != 1).sum())
        del ent, row_of, d2, has_self
    print(f"C5 200M every row: entries at >= r + eps {far}, rows without exactly one self entry {self_missing}")
    assert far == 0 and self_missing == 0
    # sampled rows against the oracle, tile by tile
    rng = np.random.default_rng(5201)
    tot, clean, angles, curv = 0, 0, [], []
    for tile in range(20):
        cx, cy = rng.uniform(-side / 2 + 5, side / 2 - 5, 2)
        near = ((xyz[:, 0] - cx).abs() < 3.0) & ((xyz[:, 1] - cy).abs() < 3.0)
        pts = torch.nonzero(near).flatten()                    # tile +- 1 m
        inner = ((xyz[pts, 0] - cx).abs() < 2.0) & ((xyz[pts, 1] - cy).abs() < 2.0)
        loc = torch.nonzero(inner).flatten()
        if loc.numel() > 10_000:
            loc = loc[torch.from_numpy(np.sort(rng.choice(loc.numel(), 10_000, replace=False))).to(ctx.device)]
        tp = xyz[pts].double()
        tree = ora.KdTree(tp.cpu().numpy())
        # rows of the tile's queries: local point indices through the tile's inverse map
        to_loc = torch.full((n,), -1, dtype=torch.int64, device=ctx.device)
        to_loc[pts] = torch.arange(pts.numel(), device=ctx.device)
        s_glob = pts[loc]
        lens_s = lens[s_glob]
        # the sampled rows as a CSR over ALL the tile's points (the others empty; loc ascends), so
        # that the checks index the offsets and the points with the same local ids
        lens_all = torch.zeros(pts.numel(), dtype=torch.int64, device=ctx.device)
        lens_all[loc] = lens_s
        sub_offs = torch.cat([torch.zeros(1, dtype=torch.int64, device=ctx.device), torch.cumsum(lens_all, 0)])
        row_of = torch.repeat_interleave(torch.arange(s_glob.numel(), device=ctx.device), lens_s)
        start = torch.cumsum(lens_s, 0) - lens_s
        pos = offs[s_glob][row_of] + (torch.arange(row_of.numel(), device=ctx.device) - start[row_of])
        sub_idx = to_loc[idx[pos].long()]
        assert bool((sub_idx >= 0).all())       # every neighbour lies inside the tile +- 1 m
        nrm_loc = torch.zeros((pts.numel(), 6), dtype=nrm.dtype, device=ctx.device)
        nrm_loc[loc] = nrm[s_glob]
        res = check_against_oracle(tree, tp, sub_offs, sub_idx, loc, loc.cpu().numpy().astype(np.int32), R,
                                   nrm=nrm_loc)
        assert res["far"] == 0 and res["dup"] == 0 and res["missing"] == 0, (tile, {k: v for k, v in res.items()
                                                                                   if np.isscalar(v)})
        tot += res["rows"]
        clean += res["clean"]
        angles.append(res["angle"])
        curv.append(res["curv_err"])
        del to_loc
    angles, curv = np.concatenate(angles), np.concatenate(curv)
    print(f"C5 200M sampled: {tot} rows from 20 tiles, {clean} band-free: {angle_summary(angles)}; "
          f"curvature err max {curv.max():.2e}")
    assert tot > 150_000 and clean > 100_000
    # the gate sits ~1.5-2x above the measured error (round 5: p99 3.2e-4, max 1.1e-3 rad), so a
    # regression that makes the fp16 normals a few times worse fails here
    assert np.percentile(angles, 99) < 5e-4 and angles.max() < 2.5e-3, angle_summary(angles)
    assert curv.max() < 5e-4
