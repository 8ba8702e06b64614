#!/usr/bin/env python3
"""Micro-benchmark of the fp64 grid kNN / normals kernels on a street scene (device ms)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudprocess_amd import ops, synth  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8_000_000)
ap.add_argument("--cells", default="0,0.05,0.08,0.12")
ap.add_argument("--ks", default="1,8,16,32")
ap.add_argument("--voxel", type=float, default=0.0, help="use voxel centroids of a 10M scene (leaf)")
args = ap.parse_args()
ctx = ops.Context(0)
xyz = synth.street_scene(args.n, 3001, device=ctx.device).to(torch.float64).contiguous()
if args.voxel > 0:
    c = torch.zeros((args.n, 6), dtype=torch.float64, device=ctx.device)
    c[:, :3] = xyz
    c[:, 3] = 1.0
    vox = ops.voxel_filter(ctx, c.view(torch.uint8).reshape(args.n, 48), args.voxel)
    xyz = vox.view(torch.float64).reshape(-1, 6)[:, :3].contiguous()
    print(f"voxel centroids: {xyz.shape[0]}, bbox {xyz.min(0).values.tolist()} {xyz.max(0).values.tolist()}")
for cs in [float(c) for c in args.cells.split(",")]:
    ix = ops.GridIndex(ctx, xyz, cell_size=cs)
    msg = [f"cell={ix.cell_size:.4f}"]
    for k in [int(v) for v in args.ks.split(",")]:
        msg.append(f"knn{k}={timed(lambda: ops.knn(ix, xyz, k)):.2f}ms")
    msg.append(f"normals32={timed(lambda: ops.normals_knn(ix, 32)):.2f}ms")
    print(" ".join(msg), flush=True)
    ix.close()
