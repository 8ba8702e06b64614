"""Timing of the exact sequential-fold centroid (fold.hip) on AoS48 clouds (profiling aid)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloudprocess_amd import ops  # noqa: E402

ctx = ops.Context(0)
for n in (1_000_000, 10_000_000, 100_000_000):
    g = torch.Generator(device="cuda").manual_seed(n)
    xyz = torch.rand((n, 3), generator=g, device="cuda", dtype=torch.float64) * 200.0 + torch.tensor(
        [431_250.0, 4_412_020.0, 30.0], device="cuda", dtype=torch.float64)
    rec = torch.zeros((n, 6), dtype=torch.float64, device="cuda")
    rec[:, :3] = xyz
    rec[:, 3] = 1.0
    cloud = rec.view(torch.uint8).view(n, 48)
    del xyz, rec
    ops.centroid(ctx, cloud)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        c, _ = ops.centroid(ctx, cloud)
    dt = (time.perf_counter() - t0) / 5
    print(f"n={n}: {dt*1e3:.3f} ms per centroid ({48*n/dt/1e9:.0f} GB/s of records)", flush=True)
    del cloud
    torch.cuda.empty_cache()
