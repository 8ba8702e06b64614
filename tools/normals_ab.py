#!/usr/bin/env python3
"""Tiled vs ring-search normals (PCP_NORMALS_TILE=0): device ms and bitwise equality of the
planes, on the C3 voxel centroids (10M street scene, leaf 0.05) or a raw street scene."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudprocess_amd import ops, synth  # noqa: E402


def timed(fn, reps=3):
    out = fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts)), out


ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--voxel", type=float, default=0.05)
ap.add_argument("--ks", default="8,32")
ap.add_argument("--tiles", default="0,1,2")
args = ap.parse_args()
ctx = ops.Context(0)
xyz = synth.street_scene(args.n, 3001, device=ctx.device).to(torch.float64).contiguous()
if args.voxel > 0:
    c = torch.zeros((args.n, 6), dtype=torch.float64, device=ctx.device)
    c[:, :3] = xyz
    c[:, 3] = 1.0
    vox = ops.voxel_filter(ctx, c.view(torch.uint8).reshape(args.n, 48), args.voxel)
    xyz = vox.view(torch.float64).reshape(-1, 6)[:, :3].contiguous()
ix = ops.GridIndex(ctx, xyz)
print(f"points {xyz.shape[0]} cell {ix.cell_size:.4f}", flush=True)
for k in [int(v) for v in args.ks.split(",")]:
    ref = None
    for t in args.tiles.split(","):
        os.environ["PCP_NORMALS_TILE"] = t
        ms, out = timed(lambda: ops.normals_knn(ix, k))
        o = out.cpu().numpy().view(np.uint32)
        same = "ref" if ref is None else ("bit-identical" if np.array_equal(o, ref) else
                                          f"DIFFER in {int((o != ref).any(axis=1).sum()) if o.ndim > 1 else int((o != ref).sum())}")
        if ref is None:
            ref = o
        print(f"k={k} tile_R={t}: {ms:.2f} ms  {same}", flush=True)
        os.environ["PCP_KNN_DEBUG"] = "1"
        ops.normals_knn(ix, k)
        torch.cuda.synchronize()
        del os.environ["PCP_KNN_DEBUG"]
