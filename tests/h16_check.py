"""Checks of C5 fp16 radius rows against exact fp64 searches (test infrastructure).

The fp16 cell-relative index can differ from the exact search only for pairs whose distance is
within EPS of r, so a row is checked by counts, all on the device:
  * every row entry lies closer than r + EPS (exact fp64 distance on the fp32 input points);
  * no row holds an entry twice;
  * the row holds as many points closer than r - EPS as the exact search finds (with the two
    checks above: every point clearly inside is there).
Rows with nothing inside the band hold exactly the exact r-neighbourhood; their F1 planes are
compared with the oracle's fp64 plane of that set, the error reported as an angle.
"""
import numpy as np
import torch

EPS = 3e-4


def row_entries(offs, idx, s):
    """(row_of, entries) of the rows of queries s (device int64): entry k of row i.  The indices
    are bounds-checked on the host first: a test indexing slip then fails this assert instead of
    faulting the device inside a gather."""
    if s.numel():
        assert int(s.min()) >= 0 and int(s.max()) < offs.numel() - 1, (int(s.min()), int(s.max()), offs.numel())
        assert int(offs[-1]) <= idx.numel(), (int(offs[-1]), idx.numel())
    lens = offs[s + 1] - offs[s]
    row_of = torch.repeat_interleave(torch.arange(s.numel(), device=s.device), lens)
    pos = offs[s][row_of] + (torch.arange(row_of.numel(), device=s.device) - (torch.cumsum(lens, 0) - lens)[row_of])
    return row_of, idx[pos].long(), lens


def band_counts(x64, offs, idx, s, r, id_to_point=None, eps=EPS):
    """far (entries at >= r + EPS), dup (repeated entries), inner (per row: entries < r - EPS),
    lens, over the rows of the queries s; x64 = the points (n, 3) fp64 on the device, indexed by
    the row entries (through id_to_point when the rows report global ids)."""
    row_of, rows, lens = row_entries(offs, idx, s)
    if rows.numel():
        lim = x64.shape[0] if id_to_point is None else id_to_point.numel()
        assert int(rows.min()) >= 0 and int(rows.max()) < lim, (int(rows.min()), int(rows.max()), lim)
    pts = rows if id_to_point is None else id_to_point[rows]
    d = torch.linalg.norm(x64[pts] - x64[s][row_of], dim=1)
    far = int((d >= r + eps).sum())
    dup = rows.numel() - torch.unique(row_of * (int(rows.max()) + 1 if rows.numel() else 1) + rows).numel()
    inner = torch.zeros(s.numel(), dtype=torch.int64, device=s.device).index_add_(0, row_of, (d < r - eps).long())
    return far, dup, inner.cpu().numpy(), lens.cpu().numpy()


def plane_angles(gp, ep):
    """Angles (rad) between the GPU planes' normals gp[:, :3] and the oracle's ep (sign-free)."""
    dots = np.clip(np.abs((gp[:, :3].astype(np.float64) * ep[:, :3]).sum(1)), 0.0, 1.0)
    return np.arccos(dots)


def oracle_planes(planes):
    return np.stack([planes[f] for f in ("normal_x", "normal_y", "normal_z", "min_value", "curvature", "distance")], 1)


def check_against_oracle(tree, x64, offs, idx, s_dev, s_local, r, nrm=None, id_to_point=None, min_rows=10, eps=EPS):
    """Band check of the rows of s_dev (device indices into x64) against the oracle kd-tree
    `tree`, whose own points s_local are the same queries.  Returns a dict of the counts and,
    with nrm, the band-free rows' plane angles and curvature errors."""
    far, dup, inner, lens = band_counts(x64, offs, idx, s_dev, r, id_to_point, eps)
    cnt_lo, _ = tree.radius_normals(s_local, r - eps)
    cnt_hi, _ = tree.radius_normals(s_local, r + eps)
    cnt_r, planes = tree.radius_normals(s_local, r)
    out = {"far": far, "dup": dup, "missing": int((inner != cnt_lo).sum()), "rows": len(s_local),
           "nbar": float(lens.mean()) if len(lens) else 0.0}
    if nrm is not None:
        clean = (cnt_lo == cnt_hi) & (lens == cnt_r) & (cnt_r >= min_rows)
        gp = nrm[s_dev].cpu().numpy()
        ep = oracle_planes(planes)
        out["clean"] = int(clean.sum())
        out["angle"] = plane_angles(gp[clean], ep[clean])
        out["curv_err"] = np.abs(gp[clean, 4] - ep[clean, 4])
    return out


def angle_summary(a):
    if not len(a):
        return "no band-free rows"
    return (f"normal angle vs oracle (rad): p50 {np.percentile(a, 50):.2e} p99 {np.percentile(a, 99):.2e} "
            f"p99.99 {np.percentile(a, 99.99):.2e} max {a.max():.2e}")
