#!/usr/bin/env python3
"""C5 pass timings (profiling aid): the count pass, the fill pass with and without the fused
normals, on the bench's 25M-point street scene (or --n).  PCP_LIB selects a library variant."""
import argparse
import math
import os
import sys

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
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=25_000_000)
    args = ap.parse_args()
    ctx = ops.Context(0)
    n = args.n
    side = math.sqrt(n / 1.5e6) * 40.0
    xyz = synth.street_scene(n, 5001, extent=(side, side), device=ctx.device)
    ix = ops.H16Index(ctx, xyz, cell_size=0.2)
    tag = os.environ.get("PCP_LIB", "default").split("/")[-2] if os.environ.get("PCP_LIB") else "default"
    t_all = timed(lambda: ix.radius_normals(0.2))
    t_rows = timed(lambda: ix.radius_normals(0.2, normals=False))
    cnt = torch.empty(n, dtype=torch.int32, device=ctx.device)
    t_cnt = timed(lambda: ctx.check(ctx.lib.pcp_h16_radius_count(ctx.h, ix.h, 0.2, n, ops._ptr(cnt))))
    print(f"{tag}: count {t_cnt:.2f} ms  count+scan+fill rows {t_rows:.2f} ms  with normals {t_all:.2f} ms", flush=True)
    ix.close()
    ctx.close()


if __name__ == "__main__":
    main()
