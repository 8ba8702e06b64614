#!/usr/bin/env python3
"""CPU model of the ICP candidate cache on a tile of the C4 bench scene at the
bench density, with the real pose sequence of the registration (the oracle's ICP iterations).

For every query and iteration it replays the engine's certificate:
  verify at pose t: settled iff  min_cached |q_t - p| < D_s - |q_t - q_s|
  search at pose t: the block around q_t certifies radius c (octant 2x2x2: distance to the faces
                    of [floor(f - 1/2), +2); 3x3x3: of [floor(f) - 1, +3)), settled iff the NN is
                    within c, and then caches the K nearest with D = min(d_{K+1}, c);
                    otherwise the fallback pass settles it and leaves D = 0 (searched again).
and counts the searched queries per iteration for several (block, K) choices, with the cost of a
search in cells scanned (8 for the octant, 27 for 3x3x3).  The verdict's question (round 3, item
3(c)): would a larger certified D from a wider iteration-0 search reduce the searched queries
summed over the 20 iterations?
  python tools/sim_icp_cache.py [n_points]
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
rmax, iters, h, mc = 0.25, 20, 0.12, 1e-3

# the registration's pose sequence (oracle correspondences + accumulators + solve)
oi = ora.F32Index(tgt)
poses, T = [], np.eye(4)
for it in range(iters):
    poses.append(T.copy())
    R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
    ei, ed = oi.correspond(q, R, t, rmax)
    acc = ora.icp_accumulate(tgt, q, R, t, ei, ed)
    rc, dT = ora.icp_solve(acc)
    T = dT @ T
print(f"{n} pts, tile {side:.1f} m; final |T - T_true| {np.abs(T - T_true).max():.2e}")

tree = cKDTree(tgt.astype(np.float64))
o = tgt.min(0).astype(np.float64)  # grid origin (bbox min)
q64 = q.astype(np.float64)


def xf(T):
    return q64 @ T[:3, :3].T + T[:3, 3]


def cert(qt, block):
    f = (qt - o) / h
    if block == "oct":
        b = np.floor(f - 0.5)
        m = np.minimum(f - b, b + 2 - f).min(1)
    else:
        c = np.floor(f)
        m = np.minimum(f - (c - 1), c + 2 - f).min(1)
    return (m - mc) * h


variants = [tuple(v.split(":")[0:1]) + (int(v.split(":")[1]),) for v in os.environ.get("SIM_VARIANTS", "oct:3,c27:3,oct:4,oct:5,oct:7,c27:7").split(",")]
Kmax = 8
for block, K in variants:
    qs = np.zeros((n, 3))          # query position at its last search
    D = np.zeros(n)                # certified bound of that search
    cache = np.zeros((n, K), np.int64)
    d3s = np.zeros(n)
    t1 = []
    searched = []
    for it, T in enumerate(poses):
        qt = xf(T)
        if it == 0:
            need = np.ones(n, bool)
        else:
            dall = np.linalg.norm(tgt[cache].astype(np.float64) - qt[:, None, :], axis=2)
            dc = dall.min(1)
            delta = np.linalg.norm(qt - qs, axis=1)
            need = ~(dc < D - delta)
            # a two-tier verify: settled from the first 3 cached points alone when their winner
            # is below min(d_3 at the search pose, D) - delta
            tier1 = dall[:, :3].min(1) < np.minimum(d3s, D) - delta
            t1.append((tier1 & ~need).sum() / max(int((~need).sum()), 1))
        idx = np.nonzero(need)[0]
        dd, ii = tree.query(qt[idx], k=K + 1, workers=8)
        c = cert(qt[idx], block)
        ok = dd[:, 0] <= c
        cache[idx] = ii[:, :K]
        d3s[idx] = dd[:, min(3, K)]
        D[idx] = np.where(ok, np.minimum(dd[:, K], c), 0.0)
        qs[idx] = qt[idx]
        searched.append(len(idx) / n)
    cells = 8 if block == "oct" else 27
    tot = sum(searched)
    print(f"{block} K={K}: searched fraction per iteration " + " ".join(f"{s:.3f}" for s in searched))
    if K > 3:
        print("   share of settled verifies settled by the first 3 cached points " + " ".join(f"{x:.2f}" for x in t1))
    print(f"   sum {tot:.3f} x n searches; iteration 0 {searched[0]:.2f}, later {tot - searched[0]:.3f}; "
          f"cells scanned per query summed {tot * cells:.1f}; cache gathers per verify {K}")
