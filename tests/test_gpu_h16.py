"""C5 (BASELINE.json configs[4]): radius r = 0.2 + normals over fp16 cell-relative
coordinates with fp32 accumulation (h16.hip).  Tolerance-based parity, as the config's
fp16 storage implies (SURVEY.md §7 hard part 6):
* neighbour sets: for every sampled query, every point closer than r - eps is in its row and
  every point of its row is closer than r + eps (eps = 3e-4 m, the fp16 offset quantisation
  bound), against an exact fp64 search (scipy cKDTree as the checker);
* normals: the row's F1 plane (calculate_feature.cpp:119-206) against a float64 PCA of the
  same row; sign canonicalised as everywhere in this build.
* multi-GPU slab + halo split (two slabs on one GPU): each slab's rows use global ids and the
  union equals the single-index result within the same band."""
import numpy as np
import pytest
import torch
from scipy.spatial import cKDTree

pytestmark = pytest.mark.gpu
R = 0.2
EPS = 3e-4


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


@pytest.fixture(scope="module")
def scene():
    from pointcloudprocess_amd import synth
    xyz = synth.street_scene(1_500_000, 5101, extent=(40.0, 40.0)).numpy()  # C5 density
    return xyz


def _check_rows(xyz, offs, idx, sample, gid_of=None):
    x64 = xyz.astype(np.float64)
    tree = cKDTree(x64)
    bad = 0
    for q in sample:
        row = idx[offs[q]:offs[q + 1]]
        d = np.linalg.norm(x64[row] - x64[q], axis=1)
        bad += int((d >= R + EPS).sum())  # nothing far outside
        near = tree.query_ball_point(x64[q], R - EPS)
        bad += len(set(near) - set(row.tolist()))  # nothing clearly inside missing
        bad += len(row) - len(set(row.tolist()))  # no duplicates
    return bad


def test_h16_radius_rows_and_normals(ctx, scene):
    from pointcloudprocess_amd import ops
    xyz = scene
    ix = ops.H16Index(ctx, torch.from_numpy(xyz).to(ctx.device), cell_size=R)
    offs, idx, nrm = ix.radius_normals(R)
    offs, idx, nrm = offs.cpu().numpy(), idx.cpu().numpy(), nrm.cpu().numpy()
    n = len(xyz)
    assert offs[0] == 0 and offs[-1] == len(idx) and (np.diff(offs) >= 1).all()  # itself included
    mean_nb = len(idx) / n
    assert 40 < mean_nb < 200, mean_nb
    rng = np.random.default_rng(7)
    sample = rng.choice(n, 4000, replace=False)
    assert _check_rows(xyz, offs, idx, sample) == 0
    # normals vs a float64 PCA of the same rows
    dots, curv = [], []
    x64 = xyz.astype(np.float64)
    for q in sample:
        row = idx[offs[q]:offs[q + 1]]
        if len(row) < 10:
            continue
        P = x64[row]
        C = np.cov((P - P.mean(0)).T, bias=True) * len(P)
        w, V = np.linalg.eigh(C)
        nv = V[:, 0]
        dots.append(abs(float(np.dot(nv, nrm[q, :3]))))
        curv.append(abs(w[0] / w.sum() - nrm[q, 4]))
    dots, curv = np.array(dots), np.array(curv)
    print(f"normals: 1-|dot| max {1 - dots.min():.3e} p99 {np.percentile(1 - dots, 99):.3e}; "
          f"curvature err max {curv.max():.3e}")
    assert np.percentile(1 - dots, 99) < 1e-6 and (1 - dots).max() < 1e-5 and curv.max() < 5e-4
    ix.close()


def test_h16_slab_halo_split_matches(ctx, scene):
    """x-slab split with an r-wide halo (SURVEY.md §8(e) for radius): rank-local rows with
    global ids == the single-index rows (band excepted)."""
    from pointcloudprocess_amd import ops
    xyz = scene
    n = len(xyz)
    cut = float(np.median(xyz[:, 0]))
    rows = {}
    for lo, hi in ((-np.inf, cut), (cut, np.inf)):
        own = np.nonzero((xyz[:, 0] >= lo) & (xyz[:, 0] < hi))[0]
        halo = np.nonzero(((xyz[:, 0] >= lo - R) & (xyz[:, 0] < lo)) | ((xyz[:, 0] >= hi) & (xyz[:, 0] < hi + R)))[0]
        gid = np.concatenate([own, halo]).astype(np.int32)
        ix = ops.H16Index(ctx, torch.from_numpy(xyz[gid]).to(ctx.device), cell_size=R)
        offs, idx, _ = ix.radius_normals(R, n_owned=len(own), global_id=torch.from_numpy(gid).to(ctx.device),
                                         normals=False)
        offs, idx = offs.cpu().numpy(), idx.cpu().numpy()
        for k in range(0, len(own), 97):
            rows[int(own[k])] = idx[offs[k]:offs[k + 1]]
        ix.close()
    keys = np.array(sorted(rows))
    x64 = xyz.astype(np.float64)
    tree = cKDTree(x64)
    bad = 0
    for q in keys:
        row = rows[q]
        d = np.linalg.norm(x64[row] - x64[q], axis=1)
        bad += int((d >= R + EPS).sum())
        bad += len(set(tree.query_ball_point(x64[q], R - EPS)) - set(row.tolist()))
    assert bad == 0 and len(keys) > 10000


def test_h16_fill_after_another_count(ctx, scene):
    """The fill takes the sorted-order row lengths its count pass kept; after a count of another
    radius in between it must gather them back from the offsets it is given -- same rows,
    same normals, byte for byte."""
    import ctypes as C
    from pointcloudprocess_amd import ops
    xyz = scene[:400_000]
    ix = ops.H16Index(ctx, torch.from_numpy(xyz).to(ctx.device), cell_size=R)
    offs, idx, nrm = ix.radius_normals(R)  # count + fill (the kept lengths)
    n = xyz.shape[0]
    lib = ctx.lib
    cnt = torch.empty(n, dtype=torch.int32, device=ctx.device)
    ctx.check(lib.pcp_h16_radius_count(ctx.h, ix.h, float(R), n, C.c_void_p(cnt.data_ptr())))
    offs2 = torch.empty(n + 1, dtype=torch.int64, device=ctx.device)
    total = C.c_int64()
    ctx.check(lib.pcp_scan_counts(ctx.h, C.c_void_p(cnt.data_ptr()), n, C.c_void_p(offs2.data_ptr()), C.byref(total)))
    cnt_b = torch.empty(n, dtype=torch.int32, device=ctx.device)  # another radius: the kept lengths change
    ctx.check(lib.pcp_h16_radius_count(ctx.h, ix.h, float(R * 0.5), n, C.c_void_p(cnt_b.data_ptr())))
    idx2 = torch.empty(max(total.value, 1), dtype=torch.int32, device=ctx.device)
    nrm2 = torch.empty((n, 6), dtype=torch.float32, device=ctx.device)
    ctx.check(lib.pcp_h16_radius_fill(ctx.h, ix.h, float(R), n, C.c_void_p(offs2.data_ptr()), None,
                                      C.c_void_p(idx2.data_ptr()), C.c_void_p(nrm2.data_ptr())))
    torch.cuda.synchronize()
    assert torch.equal(offs2.cpu(), offs.cpu())
    assert torch.equal(idx2[:total.value].cpu(), idx.cpu())
    assert torch.equal(nrm2.cpu().view(torch.int32), nrm.cpu().view(torch.int32))
    ix.close()


def test_h16_tile_matches_per_lane_kernel(ctx, scene, monkeypatch):
    """The LDS-staged row kernels (default) against the per-lane global-load kernels
    (PCP_H16_TILE=0): same rows in the same order and the same normals, byte for byte (same
    per-candidate arithmetic and visiting order); both are checked against the oracle above."""
    from pointcloudprocess_amd import ops
    out = {}
    monkeypatch.setenv("PCP_H16_CW", "0")  # the forms before the cell-wave kernels
    for mode in ("1", "0"):
        monkeypatch.setenv("PCP_H16_TILE", mode)
        ix = ops.H16Index(ctx, torch.from_numpy(scene).to(ctx.device), cell_size=R)
        offs, idx, nrm = ix.radius_normals(R)
        out[mode] = (offs.cpu(), idx.cpu(), nrm.cpu().view(torch.int32))
        ix.close()
    for a, b in zip(out["1"], out["0"]):
        assert torch.equal(a, b)


def test_h16_direct_fill_matches_staged(ctx, scene, monkeypatch):
    """The tile fill writing rows straight to caller order through its LDS row buffer
    (PCP_H16_DIRECT=1) against the staged rows + copy pass (0): byte-identical CSR and normals."""
    from pointcloudprocess_amd import ops
    out = {}
    monkeypatch.setenv("PCP_H16_CW", "0")
    monkeypatch.setenv("PCP_H16_TILE", "1")  # the direct fill is a form of the tile kernel
    for mode in ("1", "0"):
        monkeypatch.setenv("PCP_H16_DIRECT", mode)
        ix = ops.H16Index(ctx, torch.from_numpy(scene).to(ctx.device), cell_size=R)
        offs, idx, nrm = ix.radius_normals(R)
        out[mode] = (offs.cpu(), idx.cpu(), nrm.cpu().view(torch.int32))
        ix.close()
    for a, b in zip(out["1"], out["0"]):
        assert torch.equal(a, b)


def test_h16_fused_count_matches_two_pass(ctx, scene, monkeypatch):
    """The fused count (default: the count pass stages every row at a fixed stride and the planes;
    the fill moves them to caller order and redoes the rows longer than the stride) against the
    count-only pass + full fill (PCP_H16_FUSED=0): byte-identical CSR and normals, with caller
    indices and with global ids, at the default stride and at 32- and 16-entry strides (rows
    continue in spill rows until the pool runs out, the rest -- and rows longer than two strides
    -- take the redo path)."""
    import ctypes as C
    from pointcloudprocess_amd import ops
    xyz = scene[:600_000]
    n = xyz.shape[0]
    gid = torch.from_numpy(np.random.default_rng(11).permutation(n).astype(np.int32) * 3 + 5).to(ctx.device)
    lib = ctx.lib
    out = {}
    monkeypatch.setenv("PCP_H16_CW", "0")
    for mode, stride in (("0", None), ("1", None), ("1", "32"), ("1", "16")):
        monkeypatch.setenv("PCP_H16_FUSED", mode)
        if stride:
            monkeypatch.setenv("PCP_H16_FUSED_STRIDE", stride)
        else:
            monkeypatch.delenv("PCP_H16_FUSED_STRIDE", raising=False)
        ix = ops.H16Index(ctx, torch.from_numpy(xyz).to(ctx.device), cell_size=R)
        offs, idx, nrm = ix.radius_normals(R)
        idx_g = torch.empty_like(idx)
        nrm_g = torch.empty_like(nrm)
        ctx.check(lib.pcp_h16_radius_fill(ctx.h, ix.h, float(R), n, C.c_void_p(offs.data_ptr()),
                                          C.c_void_p(gid.data_ptr()), C.c_void_p(idx_g.data_ptr()),
                                          C.c_void_p(nrm_g.data_ptr())))
        torch.cuda.synchronize()
        out[(mode, stride)] = (offs.cpu(), idx.cpu(), nrm.cpu().view(torch.int32), idx_g.cpu(),
                               nrm_g.cpu().view(torch.int32))
        ix.close()
    ref = out[("0", None)]
    assert torch.equal(ref[3], gid.cpu()[ref[1].long()])
    assert torch.equal(ref[4], ref[2])
    lens = (ref[0][1:] - ref[0][:-1]).numpy()
    print(f"rows over 96: {(lens > 96).mean():.4f}, over 32 / 64: {(lens > 32).mean():.4f} / "
          f"{(lens > 64).mean():.4f}, over 16 / 32: {(lens > 16).mean():.4f} / {(lens > 32).mean():.4f}")
    for key in (("1", None), ("1", "32"), ("1", "16")):
        for a, b in zip(out[key], ref):
            assert torch.equal(a, b), key


def _radius_all(ctx, xyz, gid=None, n_owned=None):
    """count + scan + fill through the C-ABI (caller ids, and global ids when given)."""
    import ctypes as C
    from pointcloudprocess_amd import ops
    n = xyz.shape[0]
    no = n if n_owned is None else n_owned
    ix = ops.H16Index(ctx, torch.from_numpy(xyz).to(ctx.device), cell_size=R)
    offs, idx, nrm = ix.radius_normals(R, n_owned=no)
    res = [offs.cpu(), idx.cpu(), nrm.cpu()]
    if gid is not None:
        idx_g = torch.empty_like(idx)
        nrm_g = torch.empty_like(nrm)
        ctx.check(ctx.lib.pcp_h16_radius_fill(ctx.h, ix.h, float(R), no, C.c_void_p(offs.data_ptr()),
                                              C.c_void_p(gid.data_ptr()), C.c_void_p(idx_g.data_ptr()),
                                              C.c_void_p(nrm_g.data_ptr())))
        torch.cuda.synchronize()
        res += [idx_g.cpu(), nrm_g.cpu()]
    ix.close()
    return res


def _normals_close(a, b):
    """Two F1 plane arrays from the same rows with fp32 sums in different orders."""
    a, b = a.numpy().astype(np.float64), b.numpy().astype(np.float64)
    dot = np.abs((a[:, :3] * b[:, :3]).sum(1))
    ok = np.isfinite(dot)
    d = 1 - dot[ok]
    # rows of one point have 0/0 curvature in both (the F1 core's l3 / (l1 + l2 + l3))
    same_nan = bool((np.isnan(a[:, 4]) == np.isnan(b[:, 4])).all())
    fin = ok & np.isfinite(a[:, 4]) & np.isfinite(b[:, 4])
    curv = np.abs(a[fin, 4] - b[fin, 4])
    print(f"cw vs per-lane normals: 1-|dot| p99 {np.percentile(d, 99):.3e} p99.99 {np.percentile(d, 99.99):.3e} "
          f"max {d.max():.3e}; curvature diff max {curv.max():.3e}; NaN curvature rows {int(np.isnan(a[:, 4]).sum())}"
          f" (same rows: {same_nan})")
    return np.percentile(d, 99.99) < 1e-5 and curv.max() < 1e-3 and same_nan


def test_h16_cell_wave_matches_per_lane_kernel(ctx, scene, monkeypatch):
    """The cell-wave kernels (default: one wave per query cell, lanes = candidates, hits
    compacted by ballot straight into the caller CSR) against the per-lane kernel (PCP_H16_CW=0):
    the same row lengths and the same rows in the same order, byte for byte, with caller indices,
    with global ids and with an owned prefix (halo queries skipped); normals from the same rows
    with fp32 sums in another order (tree, not sequential) agree to 1e-5 in 1-|n.n'|.  The
    cloud adds a 4000-point clump inside one cell (a cell of more than 64 queries whose
    neighbourhood overflows the 384 register candidates: the segment and block loops)."""
    rng = np.random.default_rng(21)
    base = scene[:500_000]
    c0 = base[12345].astype(np.float64)
    clump = (c0 + rng.uniform(-0.04, 0.04, size=(4000, 3))).astype(np.float32)
    xyz = np.concatenate([base, clump])
    n = xyz.shape[0]
    perm = rng.permutation(n)
    xyz = xyz[perm]  # the clump spread over caller order
    gid = torch.from_numpy(rng.permutation(n).astype(np.int32) * 3 + 5).to(ctx.device)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("PCP_H16_CW", mode)
        out[mode] = (_radius_all(ctx, xyz, gid), _radius_all(ctx, xyz, n_owned=n // 3))
    (a, ah), (b, bh) = out["1"], out["0"]
    lens = (b[0][1:] - b[0][:-1]).numpy()
    print(f"rows: mean {lens.mean():.1f}, max {lens.max()}")
    assert lens.max() > 500  # the clump's rows
    for i in (0, 1, 3):
        assert torch.equal(a[i], b[i]), i
    for i in (0, 1):
        assert torch.equal(ah[i], bh[i]), ("owned", i)
    assert _normals_close(a[2], b[2]) and _normals_close(a[4], b[4]) and _normals_close(ah[2], bh[2])
    assert torch.equal(a[2].view(torch.int32), a[4].view(torch.int32))  # ids do not change the planes


@pytest.mark.parametrize("r", [0.13, 0.2])
def test_h16_cell_wave_radius_below_cell_and_tiny_clouds(ctx, scene, monkeypatch, r):
    """Cell-wave vs per-lane kernels at r < h (cells still 3x3x3, most candidates outside r) and on
    clouds of 1, 2 and 5 points (single-point rows, empty neighbour cells, planes from fewer than 3
    points): identical CSR bytes; planes equal (NaN curvature of a one-point row included)."""
    from pointcloudprocess_amd import ops
    clouds = [scene[:300_000], scene[:1], scene[:2], scene[7:12]]
    for xyz in clouds:
        out = {}
        for mode in ("1", "0"):
            monkeypatch.setenv("PCP_H16_CW", mode)
            ix = ops.H16Index(ctx, torch.from_numpy(np.ascontiguousarray(xyz)).to(ctx.device), cell_size=R)
            offs, idx, nrm = ix.radius_normals(r)
            out[mode] = (offs.cpu(), idx.cpu(), nrm.cpu())
            ix.close()
        a, b = out["1"], out["0"]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), len(xyz)
        if len(xyz) < 10:
            assert torch.allclose(a[2], b[2], atol=1e-6, equal_nan=True), (len(xyz), a[2], b[2])
        else:
            assert _normals_close(a[2], b[2])


def test_h16_cell_wave_dropped_points(ctx, scene, monkeypatch):
    """Non-finite points are dropped by the build: their rows stay empty and their planes keep the
    default, in the cell-wave path (which skips the clears when nothing was dropped) as in the
    per-lane one."""
    from pointcloudprocess_amd import ops
    xyz = np.ascontiguousarray(scene[:50_000]).copy()
    xyz[[3, 777, 4000]] = np.nan
    xyz[12345, 1] = np.inf
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("PCP_H16_CW", mode)
        ix = ops.H16Index(ctx, torch.from_numpy(xyz).to(ctx.device), cell_size=R)
        offs, idx, nrm = ix.radius_normals(R)
        out[mode] = (offs.cpu(), idx.cpu(), nrm.cpu())
        ix.close()
    a, b = out["1"], out["0"]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    lens = a[0][1:] - a[0][:-1]
    for k in (3, 777, 4000, 12345):
        assert int(lens[k]) == 0
        assert torch.equal(a[2][k], torch.tensor([0.0, 0.0, 0.0, 0.0, 1.0, 0.0]))
    assert _normals_close(a[2], b[2])
