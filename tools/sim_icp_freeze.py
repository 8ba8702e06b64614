#!/usr/bin/env python3
"""CPU model: how many queries could leave the verify pass for good (a per-query "freeze": its
winner cannot change while the pose moves less than half its margin) if the whole future motion
of the registration were known in advance (hindsight upper bound).  Tile of the C4 scene at the
bench density, the oracle registration's own poses.  python tools/sim_icp_freeze.py"""
import os, sys, math, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import oracle_ctypes as ora
from pointcloudprocess_amd import synth
from scipy.spatial import cKDTree
n = 2_000_000
side = 200.0 * math.sqrt(n / 50e6)
T_true = synth.rigid()
tgt, q = synth.icp_pair(n, n, 4001, 4002, T_true, extent=(side, side))
tgt, q = tgt.numpy(), q.numpy()
rmax, iters = 0.25, 20
oi = ora.F32Index(tgt)
poses, T = [], np.eye(4)
for it in range(iters):
    poses.append(T.copy())
    R, t = T[:3, :3].astype(np.float32), T[:3, 3].astype(np.float32)
    ei, ed = oi.correspond(q, R, t, rmax)
    acc = ora.icp_accumulate(tgt, q, R, t, ei, ed)
    rc, dT = ora.icp_solve(acc)
    T = dT @ T
q64 = q.astype(np.float64)
tree = cKDTree(tgt.astype(np.float64))
# max displacement over the whole query set between pose a and pose b (50 m tile -> scale to 200 m: x4 lever arm)
def xf(T): return q64 @ T[:3, :3].T + T[:3, 3]
Q = [xf(T) for T in poses]
# hindsight future-motion bound after iteration t: max over t' > t of max_i |q_t' - q_t|
M = []
for t in range(iters):
    m = 0.0
    for t2 in range(t + 1, iters):
        m = max(m, np.linalg.norm(Q[t2] - Q[t], axis=1).max())
    M.append(m)
print("future motion bound per iteration (mm):", " ".join(f"{1e3*m:.2f}" for m in M))
# per-query gap at each iteration: (2nd nearest - nearest) at the current pose (exact NN, a proxy for
# the cached set's winner margin and D)
frozen = np.zeros(n, bool)
for t in range(iters):
    dd, ii = tree.query(Q[t], k=2, workers=8)
    gap = dd[:, 1] - dd[:, 0]
    newly = (~frozen) & (gap > 2 * M[t]) & (dd[:, 0] <= rmax)
    print(f"iter {t}: active {(~frozen).mean():.3f}, newly frozen {newly.mean():.3f}")
    frozen |= newly
