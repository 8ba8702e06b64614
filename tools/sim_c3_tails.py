#!/usr/bin/env python3
"""CPU model (round 6): where the C3 normals' uncertified rows live.

The C3 step's normals end in two tail passes over the rows the tile cannot certify: the near
pass (a Chebyshev-3 row window per row) and the far pass (brick shells, one wave per row).  Both
run on a nearly idle GPU after the tile.  If those rows concentrate in sparse query bricks, the
tile could take the sparse bricks first and run their tails on a second stream under the rest of
the tile.  This model builds a C3-like centroid cloud (street scene, 0.05 m voxel centroids),
takes every point's exact 32nd-neighbour distance (scipy kd-tree) and classifies the rows as the
tile's window bound would (R = 2 cells) and as the near pass's (R = 3), then reports the share of
rows and of tail rows per 8x8x8-cell brick occupancy class.
  python tools/sim_c3_tails.py [n_points] [cell]
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pointcloudprocess_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
h = float(sys.argv[2]) if len(sys.argv) > 2 else 0.192  # the C3 index's automatic cell size (GPU)
xyz = synth.street_scene(n, 3001).numpy().astype(np.float64)
key = np.floor((xyz - xyz.min(0)) / 0.05).astype(np.int64)
k1 = (key[:, 2] * 8192 + key[:, 1]) * 8192 + key[:, 0]
_, inv, cnt = np.unique(k1, return_inverse=True, return_counts=True)
cent = np.stack([np.bincount(inv, xyz[:, a]) / cnt for a in range(3)], 1)
m = len(cent)
print(f"{n} pts -> {m} centroids, cell {h}")
tree = cKDTree(cent)
d32 = np.empty(m)
for s in range(0, m, 1_000_000):
    d, _ = tree.query(cent[s:s + 1_000_000], k=32, workers=8)
    d32[s:s + 1_000_000] = d[:, 31]
f = (cent - cent.min(0)) / h
c = np.floor(f)
fr = f - c
face = np.minimum(fr, 1 - fr).min(1)
tile_fail = d32 > (2 + face) * h  # beyond the R = 2 window's faces
far = d32 > (3 + face) * h        # beyond the near pass's Chebyshev-3 window
b = (c // 8).astype(np.int64)
bk = (b[:, 2] * 4096 + b[:, 1]) * 4096 + b[:, 0]
_, binv, bcnt = np.unique(bk, return_inverse=True, return_counts=True)
occ = bcnt[binv]
print(f"rows beyond the tile's window: {tile_fail.sum()} ({tile_fail.mean():.4%}); beyond the near window: {far.sum()}")
print("brick occupancy <= T: share of rows | of tile-deferred rows | of far rows")
for T in (16, 32, 64, 128, 256, 512, 1024):
    sel = occ <= T
    print(f"  T={T:5d}: {sel.mean():.4f} | {tile_fail[sel].sum() / max(1, tile_fail.sum()):.3f} | "
          f"{far[sel].sum() / max(1, far.sum()):.3f}")
