#!/usr/bin/env python3
"""CPU model (round 6): could verify gather only the cached winner? With the gap g = d(2nd) - d(1st)
among the cached points at the search pose, the winner is unchanged while |q_t - q_s| < g / 2, so the
other two gathers could be skipped.  Prints, per launch, the share of settled queries the rule covers.
  python tools/sim_icp_gap.py [n_points]
"""
import math
import os
import sys

import numpy as np
from scipy.spatial import cKDTree
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
import oracle_ctypes as ora
from pointcloudprocess_amd import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
side = 200.0 * math.sqrt(n / 50e6)
T_true = synth.rigid()
tgt, q = synth.icp_pair(n, n, 4001, 4002, T_true, extent=(side, side))
tgt, q = tgt.numpy(), q.numpy()
rmax, iters, h, mc = 0.25, 20, 0.12, 1e-3
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
q64 = q.astype(np.float64); t64 = tgt.astype(np.float64)
def cert(qt):
    f = (qt - o) / h; b = np.floor(f - 0.5); m = np.minimum(f - b, b + 2 - f).min(1); return (m - mc) * h
K = 3
qs = np.zeros((n, 3)); D = np.zeros(n); cache = np.zeros((n, K), np.int64); gap = np.zeros(n)
for it, T in enumerate(poses):
    qt = q64 @ T[:3, :3].T + T[:3, 3]
    if it == 0:
        need = np.ones(n, bool); settled_gap = None
    else:
        delta = np.linalg.norm(qt - qs, axis=1)
        dall = np.linalg.norm(t64[cache] - qt[:, None, :], axis=2)
        need = ~(dall.min(1) < D - delta)
        st = ~need
        g1 = delta < gap / 2
        print(f"launch {it}: settled {st.mean():.3f}; of them winner fixed by gap rule {(g1 & st).sum() / max(1, st.sum()):.3f}; median delta {np.median(delta)*1e3:.3f} mm")
    idx = np.nonzero(need)[0]
    dd, ii = tree.query(qt[idx], k=K + 1, workers=8)
    c = cert(qt[idx]); ok = dd[:, 0] <= c
    cache[idx] = ii[:, :K]
    gap[idx] = dd[:, 1] - dd[:, 0]
    D[idx] = np.where(ok, np.minimum(dd[:, K], c), 0.0)
    qs[idx] = qt[idx]
