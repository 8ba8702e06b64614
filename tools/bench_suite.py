#!/usr/bin/env python3
"""Secondary benchmarks of the hot path (BASELINE.json configs C1, C2, C3, C5-radius).

bench.py measures the headline C4 (ICP) line; this prints one JSON line per config with
the same roofline convention (algorithmic bytes or flops per launch over
the launch's device time).  Inputs are resident in HBM before timing; device time comes
from events on the stream the kernels run on (the torch current stream, which the
libpcp context uses).

  python tools/bench_suite.py [--only c2,c3,...] [--reps 3] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from pointcloudprocess_amd import ops, synth  # noqa: E402

HBM_GBS = 8000.0
CPU_THREADS = min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
os.environ["OMP_NUM_THREADS"] = str(CPU_THREADS)  # the box's CPU share for one GPU
F32_MFMA_TFS = 157.3


def timed(fn, reps):
    """Median device ms of fn() over reps (events on the current stream), after 1 warmup."""
    fn()
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


def cpu_time(fn):
    t0 = time.perf_counter()
    r = fn()
    return time.perf_counter() - t0, r


def c2(ctx, args):
    n = args.c2_n
    t = synth.uniform_cube(n, 2001, half=50.0, device=ctx.device)
    q = synth.uniform_cube(n, 2002, half=50.0, device=ctx.device)
    ms, _ = timed(lambda: ops.knn_bruteforce(ctx, t, q, 8), args.reps)
    fb = ops.knn_bruteforce_last_fallback(ctx)
    flops = 8.0 * n * n
    line = {"config": "C2", "workload": f"brute-force kNN k=8, {n}x{n} uniform [-50,50]^3",
            "ms": round(ms, 3), "value": round(n / ms / 1e3, 3), "unit": "Mqueries/s",
            "roofline": {"bound": "mfma", "achieved": round(flops / ms / 1e9, 2), "peak": F32_MFMA_TFS,
                         "unit": "TFLOP/s", "frac": round(flops / ms / 1e9 / F32_MFMA_TFS, 4)},
            "fallback_queries": fb}
    if not args.no_cpu:
        import oracle_ctypes as ora
        tc = t.cpu().numpy()
        qs = q[: args.cpu_q].cpu().numpy()
        dt, _ = cpu_time(lambda: ora.KdTree(tc).knn(qs, 8))
        line["cpu_baseline"] = {"value": round(len(qs) / dt / 1e6, 3), "unit": "Mqueries/s", "cores": CPU_THREADS,
                                "kind": "port", "sample": f"oracle kd-tree build over {n} + {len(qs)} queries"}
    return line


def street_aos(n, seed, device):
    xyz = synth.street_scene(n, seed, device=device).to(torch.float64)
    c = torch.zeros((n, 6), dtype=torch.float64, device=device)
    c[:, :3] = xyz
    c[:, 3] = 1.0
    g = torch.Generator(device=device)
    g.manual_seed(seed + 7)
    rgba = torch.randint(0, 2**31 - 1, (n,), generator=g, device=device, dtype=torch.int64)
    stamp = torch.arange(n, device=device, dtype=torch.int64) // 100000
    c[:, 4] = (rgba | (stamp << 32)).view(torch.float64)
    return c.view(torch.uint8).reshape(n, 48).contiguous(), xyz


def c3(ctx, args):
    n = args.c3_n
    cloud, xyz = street_aos(n, 3001, ctx.device)
    ms_v, out = timed(lambda: ops.voxel_filter(ctx, cloud, 0.05), args.reps)
    m = out.shape[0]
    vbytes = n * (24 + 8) + 48 * m
    lines = [{"config": "C3-voxel", "workload": f"VoxelGrid leaf 0.05f on {n} street-scene pts -> {m} voxels",
              "ms": round(ms_v, 3), "value": round(n / ms_v / 1e3, 3), "unit": "Mpoints/s",
              "roofline": {"bound": "hbm", "achieved": round(vbytes / ms_v / 1e6, 2), "peak": HBM_GBS,
                           "unit": "GB/s", "frac": round(vbytes / ms_v / 1e6 / HBM_GBS, 4)}}]
    vox = ops.cloud_to_host(out)
    vx = torch.from_numpy(np.stack([vox["x"], vox["y"], vox["z"]], 1)).to(ctx.device)
    ms_b, ix = timed(lambda: ops.GridIndex(ctx, vx), 1)
    ms_n, _ = timed(lambda: ops.normals_knn(ix, 32), args.reps)
    nbytes = m * (12 + 16)
    lines.append({"config": "C3-normals", "workload": f"kNN(32) PCA normals over the {m} voxel centroids",
                  "ms": round(ms_n, 3), "index_build_ms": round(ms_b, 3), "value": round(m / ms_n / 1e3, 3),
                  "unit": "Mpoints/s",
                  "roofline": {"bound": "hbm", "achieved": round(nbytes / ms_n / 1e6, 2), "peak": HBM_GBS,
                               "unit": "GB/s", "frac": round(nbytes / ms_n / 1e6 / HBM_GBS, 4)}})
    if not args.no_cpu:
        import oracle_ctypes as ora
        s = args.cpu_pts
        host = ops.cloud_to_host(cloud[:s])
        dt, _ = cpu_time(lambda: ora.voxel_filter(host, 0.05))
        lines[0]["cpu_baseline"] = {"value": round(s / dt / 1e6, 3), "unit": "Mpoints/s", "cores": 1, "kind": "port",
                                    "sample": f"oracle voxel filter on the first {s} points"}
        vs = vx[: args.cpu_pts // 4].cpu().numpy()
        dt, _ = cpu_time(lambda: ora.normals_knn(vs, 32))
        lines[1]["cpu_baseline"] = {"value": round(len(vs) / dt / 1e6, 3), "unit": "Mpoints/s",
                                    "cores": CPU_THREADS, "kind": "port",
                                    "sample": f"oracle kd-tree normals k=32 on {len(vs)} voxel centroids"}
    return lines


def c5(ctx, args):
    n = args.c5_n
    xyz = synth.street_scene(n, 5001, device=ctx.device).to(torch.float64).contiguous()
    ix = ops.GridIndex(ctx, xyz)
    ms, (offs, idx, d2) = timed(lambda: ops.radius(ix, xyz, 0.2), args.reps)
    nbar = idx.numel() / n
    byts = n * (24 + 8) + idx.numel() * 12
    return {"config": "C5-radius", "workload": f"radiusSearch r=0.2 of all {n} street-scene pts (1 GPU slice)",
            "ms": round(ms, 3), "value": round(n / ms / 1e3, 3), "unit": "Mqueries/s", "nbar": round(nbar, 2),
            "roofline": {"bound": "hbm", "achieved": round(byts / ms / 1e6, 2), "peak": HBM_GBS, "unit": "GB/s",
                         "frac": round(byts / ms / 1e6 / HBM_GBS, 4)}}


def c1(ctx, args):
    rng = np.random.default_rng(1001)
    base = rng.uniform(-10, 10, (100_000, 3)).astype(np.float32).astype(np.float64)
    dup = base[rng.integers(0, len(base), 5000)]
    pts = np.concatenate([base, dup])
    import oracle_ctypes as ora
    cloud = ops.cloud_to_device(ora.make_cloud(pts), ctx.device)
    q = torch.from_numpy(np.random.default_rng(1002).uniform(-10, 10, (100_000, 3))).to(ctx.device)

    def run():
        vox = ops.voxel_filter(ctx, cloud, 0.1)
        ix = ops.GridIndex(ctx, vox)
        return ops.knn(ix, q, 1)
    ms, _ = timed(run, args.reps)
    return {"config": "C1", "workload": "voxel(0.1) of 105k pts + index + 1-NN of 100k queries",
            "ms": round(ms, 3), "value": round(105_000 / ms / 1e3, 3), "unit": "Mpoints/s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c2,c3,c5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--c2-n", type=int, default=1_000_000)
    ap.add_argument("--c3-n", type=int, default=10_000_000)
    ap.add_argument("--c5-n", type=int, default=25_000_000)
    ap.add_argument("--cpu-q", type=int, default=200_000)
    ap.add_argument("--cpu-pts", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    ctx = ops.Context(0)
    for name in args.only.split(","):
        r = {"c1": c1, "c2": c2, "c3": c3, "c5": c5}[name](ctx, args)
        for line in (r if isinstance(r, list) else [r]):
            print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
