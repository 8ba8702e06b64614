"""Micro-benchmark of one ICP correspondence iteration (profiling aid, not part of the
product).  Builds the C4 workload once, then times a host-loop registration (pcp_icp_step +
host solve per iteration) from the identity; set
PCP_ICP_ABLATE=<flags> to time ablated kernels (results are then meaningless)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudprocess_amd import ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=50_000_000)
ap.add_argument("--cell", type=float, default=0.12)
ap.add_argument("--rmax", type=float, default=0.25)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()

ctx = ops.Context(0)
T_true = synth.rigid()
tgt, q = synth.icp_pair(args.n, args.n, 4001, 4002, T_true, device=ctx.device)
torch.cuda.synchronize()
t0 = time.perf_counter()
index = ops.GridIndex(ctx, tgt, cell_size=args.cell)
icp = ops.ICP(index, q)
torch.cuda.synchronize()
print(f"build+sort {1e3 * (time.perf_counter() - t0):.1f} ms  cells {ctx.lib.pcp_index_cells(index.h)}", flush=True)
ap2 = None
for rep in range(args.reps):
    T = np.eye(4)
    tot = 0.0
    for it in range(args.iters):
        acc = icp.step(T, args.rmax)
        ms, _ = icp.last_kernel_ms()
        tot += ms
        rc, dT = ops.icp_solve(acc.cpu().numpy())
        print(f"rep{rep} iter{it}: {ms:.4f} ms  fallback {icp.last_fallback()}", flush=True)
        if rc != 0:
            break
        Tn = dT @ T
        # largest displacement this update causes over the scene's box (corners at +-100 m, z 0..20)
        cs = np.array([[x, y, z, 1.0] for x in (-100, 100) for y in (-100, 100) for z in (0, 20)])
        disp = np.abs((cs @ (Tn - T).T)[:, :3]).max()
        print(f"   pose step max corner displacement {disp * 1e3:.3f} mm", flush=True)
        T = Tn
    print(f"rep{rep}: {tot:.3f} ms over {args.iters} iterations ({tot / args.iters:.4f} ms/iter)  "
          f"|T-T_true| {np.abs(T - T_true).max():.2e}", flush=True)
