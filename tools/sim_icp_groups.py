#!/usr/bin/env python3
"""CPU model (round-5 verdict item 1(a)): would scoring the search lists block-by-block on the
matrix cores pay?  On a tile of the C4 bench scene at the bench density, with the registration's
real pose sequence and the engine's cache certificate (as tools/sim_icp_cache.py, octant block,
3 cached points), it takes each launch's searched queries and compares, per launch:

  octant   the current search: each searched query scans its own 2x2x2 octant block
           (targets in the 8 cells at floor(f - 1/2));
  group    the listed queries grouped by 2x2x2 group of octant-block origins (so their octant
           blocks lie in one 3x3x3 cell neighbourhood), each group's queries scored against the
           whole neighbourhood: m x C pairs for m listed queries and C targets;
  tiled    the same on 16 x 16 MFMA tiles: ceil(m / 16) * 16 x ceil(C / 16) * 16 scores;
  cw64     the verdict's variant: queries grouped by 2x2x2 cells, scored against the 4x4x4 cells
           around them, on 16 x 16 tiles.

The inflation is (scores per searched query) / (octant candidates per searched query).  The
verdict's criterion: build the block-MFMA search only if it is <= 3x.

Round 6 (verdict item 1(a)): the C5 cell-wave form, counted in WAVE PASSES (one wave-wide step
that evaluates one 64-lane slice of candidates against one query set) per listed query:
  lanes    the current form: chunks of 64 / G consecutive listed queries (list order = sorted
           order), G lanes per query by the device density rule (G = 1 above 36 %, 2 above 8 %,
           else 4), each chunk ceil(Lw / G) steps with Lw the chunk's longest octant list;
  cellwave one wave per 2x2x2 query brick (bricks of octant-block origins) holding >= 1 listed
           query: its 3x3x3-cell neighbourhood loaded once (ceil(C / 64) coalesced steps), then
           per listed query (wave-uniform) ceil(C / 64) evaluation steps plus the wave-wide
           top-3 merge of 6 butterfly stages (counted as 6 / 4 = 1.5 passes: ~4 DPP ops per
           stage against ~16 VALU ops of a candidate step) and a per-brick set-up of 1 pass.
  python tools/sim_icp_groups.py [n_points]
"""
import math
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ctypes as ora  # noqa: E402  (test infrastructure: the reference ICP poses)
from pointcloudprocess_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
side = 200.0 * math.sqrt(n / 50e6)
T_true = synth.rigid()
tgt, q = synth.icp_pair(n, n, 4001, 4002, T_true, extent=(side, side))
tgt, q = tgt.numpy(), q.numpy()
rmax, iters, h, mc, K = 0.25, 20, 0.12, 1e-3, 3

oi = ora.F32Index(tgt)
poses, T = [], np.eye(4)
for it in range(iters):
    poses.append(T.copy())
    R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
    ei, ed = oi.correspond(q, R, t, rmax)
    acc = ora.icp_accumulate(tgt, q, R, t, ei, ed)
    rc, dT = ora.icp_solve(acc)
    T = dT @ T

tree = cKDTree(tgt.astype(np.float64))
o = tgt.min(0).astype(np.float64)
q64 = q.astype(np.float64)
# target counts per cell (hash of the integer cell coordinates)
tc = np.floor((tgt.astype(np.float64) - o) / h).astype(np.int64) + 4
M = int(tc.max()) + 8
key = (tc[:, 2] * M + tc[:, 1]) * M + tc[:, 0]
uk, cnt = np.unique(key, return_counts=True)


def cell_count(c):  # c: (m, 3) integer cells (grid-shifted by +4) -> targets in each
    k = (c[:, 2] * M + c[:, 1]) * M + c[:, 0]
    i = np.searchsorted(uk, k)
    i[i >= len(uk)] = 0
    return np.where(uk[i] == k, cnt[i], 0)


def box_count(lo, w):  # targets in the w x w x w cells from lo (m, 3)
    tot = np.zeros(len(lo), np.int64)
    for dz in range(w):
        for dy in range(w):
            for dx in range(w):
                tot += cell_count(lo + np.array([dx, dy, dz]))
    return tot


def grouped(keys, per_group_cands, tile):
    """scores for the groups of `keys` (one per listed query): m x C or tiled."""
    g, inv, m = np.unique(keys, axis=0, return_inverse=True, return_counts=True)
    C = per_group_cands(g)
    if tile:
        return float((np.ceil(m / 16) * 16 * np.ceil(C / 16) * 16).sum())
    return float((m * C).sum())


qs_ = np.zeros((n, 3))
D = np.zeros(n)
cache = np.zeros((n, K), np.int64)
print(f"{n} pts, tile {side:.1f} m")
print("launch  searched  octant/q  group m*C/q  infl  tiled/q  infl  cw64-tiled/q  infl")
tot = {"oct": 0.0, "grp": 0.0, "til": 0.0, "cw": 0.0, "q": 0, "wl": 0.0, "wc": 0.0}
wave_rows = []
for it, T in enumerate(poses):
    qt = q64 @ T[:3, :3].T + T[:3, 3]
    if it == 0:
        need = np.ones(n, bool)
    else:
        dall = np.linalg.norm(tgt[cache].astype(np.float64) - qt[:, None, :], axis=2)
        need = ~(dall.min(1) < D - np.linalg.norm(qt - qs_, axis=1))
    idx = np.nonzero(need)[0]
    dd, ii = tree.query(qt[idx], k=K + 1, workers=8)
    f = (qt[idx] - o) / h
    b = np.floor(f - 0.5).astype(np.int64) + 4                    # octant block origin (shifted)
    m_ = np.minimum(f - (b - 4), (b - 4) + 2 - f).min(1)
    c_ = (m_ - mc) * h
    ok = dd[:, 0] <= c_
    cache[idx] = ii[:, :K]
    D[idx] = np.where(ok, np.minimum(dd[:, K], c_), 0.0)
    qs_[idx] = qt[idx]
    oct_c = float(box_count(b, 2).sum())
    grp = grouped(b // 2, lambda g: box_count(g * 2, 3), False)
    til = grouped(b // 2, lambda g: box_count(g * 2, 3), True)
    cell = np.floor(f).astype(np.int64) + 4
    cw = grouped(cell // 2, lambda g: box_count(g * 2 - 1, 4), True)
    nq_ = len(idx)
    # wave passes: the current lanes form over the list in sorted order (queries are sorted by the
    # brick-major key of their octant block, so sort the listed queries by it)
    G = 1 if nq_ * 100 > n * 36 else (2 if nq_ * 100 > n * 8 else 4)
    L = box_count(b, 2)
    ordk = np.lexsort((b[:, 0] % 8, b[:, 1] % 8, b[:, 2] % 8, b[:, 0] // 8, b[:, 1] // 8, b[:, 2] // 8))
    Ls = L[ordk]
    qpc = 64 // G
    nch = -(-nq_ // qpc)
    Lp = np.zeros(nch * qpc, np.int64)
    Lp[:nq_] = Ls
    Lw = Lp.reshape(nch, qpc).max(1)
    w_lanes = float(np.ceil(Lw / G).sum())
    gb, ginv, gm = np.unique(b // 2, axis=0, return_inverse=True, return_counts=True)
    C = box_count(gb * 2, 3)
    steps = np.ceil(C / 64)
    w_cell = float((steps + 1.0 + gm * (steps + 1.5)).sum())
    tot["wl"] += w_lanes
    tot["wc"] += w_cell
    wave_rows.append((it, nq_ / n, G, w_lanes / nq_, len(gb), nq_ / len(gb), float(C.mean()), w_cell / nq_))
    tot["oct"] += oct_c
    tot["grp"] += grp
    tot["til"] += til
    tot["cw"] += cw
    tot["q"] += nq_
    print(f"{it:6d}  {nq_ / n:8.3f}  {oct_c / nq_:8.1f}  {grp / nq_:11.1f}  {grp / oct_c:4.1f}  {til / nq_:7.1f}  "
          f"{til / oct_c:4.1f}  {cw / nq_:12.1f}  {cw / oct_c:4.1f}")
print("\nwave passes per listed query (verdict r5 item 1(a))")
print("launch  searched  G  lanes/q  bricks  q/brick  C/brick  cellwave/q  ratio")
for (it, fr, G, wl, nb, qb, cb, wc) in wave_rows:
    print(f"{it:6d}  {fr:8.3f}  {G}  {wl:7.3f}  {nb:6d}  {qb:7.2f}  {cb:7.1f}  {wc:10.3f}  {wc / wl:5.1f}")
print(f"launches 1-19: lanes {sum(r[3] * r[1] for r in wave_rows[1:]) / sum(r[1] for r in wave_rows[1:]):.3f}, "
      f"cellwave {sum(r[7] * r[1] for r in wave_rows[1:]) / sum(r[1] for r in wave_rows[1:]):.3f} wave passes per listed query")
print(f"all launches: octant {tot['oct'] / tot['q']:.1f} candidates per searched query; group m*C x{tot['grp'] / tot['oct']:.2f}, "
      f"16x16-tiled x{tot['til'] / tot['oct']:.2f}, cw64 tiled x{tot['cw'] / tot['oct']:.2f}")
