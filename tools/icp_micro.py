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
        T = dT @ T
    print(f"rep{rep}: {tot:.3f} ms over {args.iters} iterations ({tot / args.iters:.4f} ms/iter)  "
          f"|T-T_true| {np.abs(T - T_true).max():.2e}", flush=True)
