"""bench.py --config C1 | C2 | C3 | C5: the other BASELINE.json configs, one JSON line each with
the bench.py contract (value = whole-job throughput over the timed steps, max over ranks;
roofline of the dominant kernel from HIP events on the stream it runs on; cpu_baseline = the
oracle restatement on a bounded sample, rank 0 at N = 1 only).  Every rank runs its own batch
(weak scaling, no collective).  Inputs are resident in HBM before the timed region.

Algorithmic bytes / flops per unit follow SURVEY.md §8(d):
  C2  8 flops per (query, target) pair (the K=4 contraction) -> fp32 MFMA peak
  C3  voxel: 32 B read per point + 48 B per voxel written; normals: 12 B read + 16 B written per
      centroid (the dominant kernel)
  C5  6 B (fp16 xyz) + 4 B per neighbour index + 16 B (normal, curvature) + 4 B (CSR offset) per point
"""
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
F32_MFMA_TFS = 157.3       # MI355X_MICROARCH.md: dense fp32 MFMA (= fp32 vector) peak


class Timer:
    """HIP events on the torch current stream (the stream libpcp's context launches on)."""

    def __init__(self):
        self.ms = 0.0
        self.n = 0

    def __call__(self, fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        torch.cuda.synchronize()
        self.ms += s.elapsed_time(e)
        self.n += 1
        return out

    @property
    def avg(self):
        return self.ms / max(self.n, 1)


_ORA = {}

# the kernels each config's timed call runs (their PMC traffic is the line's roofline.traffic)
PMC_KERNELS = {
    "C2": ("knn_bf.hip", ("k_bf_mfma", "k_bf_fallback", "k_bf_targets", "k_bf_pad")),
    "C3": ("knn.hip", ("k_normals_tile", "k_normals", "k_normals_coop", "k_brick_keys", "k_plane_default")),
    "C5": ("h16.hip", ("k_h16_mx", "k_h16_mx_planes", "k_h16_mx_planes_fb", "tile_scan", "k_h16_ids",
                       "k_h16_plane_default")),
}


def pmc_traffic(cfg, workload, calls=1):
    """HBM bytes per timed call (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction)
    of the config's kernels, from the newest profiles/*/pmc_traffic_<cfg>.json measured on the
    current source of those kernels (sha1 match) and on this run's workload (its "workload" record
    equals `workload`: points per rank, world size, split), else None.  Made by tools/pmc_summary.py
    --src=<file> --key=... from separate FETCH_SIZE / WRITE_SIZE passes of `bench.py --config <cfg>
    --steps 1 --warmup 0 --no-cpu` (one timed call)."""
    import glob
    import hashlib
    src, kernels = PMC_KERNELS[cfg]
    sha = hashlib.sha1(open(os.path.join(ROOT, "pointcloudprocess_amd", "csrc", src), "rb").read()).hexdigest()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_traffic_{cfg}.json")), key=os.path.getmtime,
                    reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("src_sha1") != sha or d.get("workload") != workload:
            continue
        tot = 0.0
        for k in kernels:
            e = d["kernels"].get(k)
            if e is not None:
                tot += e["launches"] * (e["fetch_bytes_avg"] + (e["write_bytes_avg"] or 0.0))
        return tot / calls, os.path.relpath(f, ROOT)
    return None


def _with_traffic(roof, cfg, workload):
    t = pmc_traffic(cfg, workload)
    if roof is not None and t is not None:
        roof["traffic"] = round(t[0] / (roof["kernel_avg_ms"] * 1e-3) / 1e9, 2)
        roof["traffic_bytes_per_launch"] = round(t[0])
        roof["traffic_source"] = t[1]
    elif roof is not None:
        roof["traffic"] = None
        roof["traffic_source"] = f"none: no sha-matched PMC record of this workload {workload}"
    return roof


def _oracle():
    """The oracle built -O3 -march=native on this host (bench.native_oracle); cpu legs only."""
    if not _ORA:
        import bench
        _ORA["ora"], _ORA["build"] = bench.native_oracle()
    return _ORA["ora"]


def _thread_options():
    """Thread counts the CPU legs try: every CPU of the process's affinity set, and that count
    capped at the cgroup CPU quota when there is one.  Which is faster depends on the leg (on
    the GPU box, 256 affinity CPUs share a 16-CPU quota: the C4 leg ran 3x slower at 256
    threads, the brute-force C2 leg 2x faster), so each leg reports the faster."""
    import bench
    naff = len(os.sched_getaffinity(0))
    quota = bench.cpu_info()[3]
    cap = max(1, min(naff, int(quota))) if quota else naff
    return sorted({cap, naff})


def _fastest(run):
    """(seconds, threads, {threads: seconds}) of run(nthreads) over _thread_options()."""
    times = {}
    for th in _thread_options():
        t0 = time.perf_counter()
        run(th)
        times[th] = time.perf_counter() - t0
    th = min(times, key=times.get)
    return times[th], th, {k: round(v, 3) for k, v in times.items()}


def _cpu_meta(rec):
    import bench
    model, ncpu, naff, quota = bench.cpu_info()
    rec.update({"build": _ORA.get("build"), "cores_all": naff, "nproc": ncpu, "affinity_cpus": naff,
                "cgroup_cpu_quota": quota, "cpu_model": model})
    return rec


def street_aos48(n, seed, device):
    """PointXYZRGBA-layout (48 B) street scene: xyz fp64, data[3] = 1, rgba + stamp_id."""
    xyz = __import__("pointcloudprocess_amd.synth", fromlist=["synth"]).street_scene(n, seed, device=device)
    c = torch.zeros((n, 6), dtype=torch.float64, device=device)
    c[:, :3] = xyz.to(torch.float64)
    c[:, 3] = 1.0
    g = torch.Generator(device=device)
    g.manual_seed(seed + 7)
    rgba = torch.randint(0, 2**31 - 1, (n,), generator=g, device=device, dtype=torch.int64)
    stamp = torch.arange(n, device=device, dtype=torch.int64) // 100000
    c[:, 4] = (rgba | (stamp << 32)).view(torch.float64)
    return c.view(torch.uint8).reshape(n, 48).contiguous()


def run_steps(step, steps, warmup, barrier):
    for _ in range(warmup):
        step(False)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    torch.cuda.synchronize()
    barrier()
    return time.perf_counter() - t0


def cfg_c1(ctx, args, rank, timer):
    from pointcloudprocess_amd import ops
    rng = np.random.default_rng(1001 + rank)
    base = rng.uniform(-10, 10, (100_000, 3)).astype(np.float32).astype(np.float64)
    pts = np.concatenate([base, base[rng.integers(0, len(base), 5000)]])
    cloud = np.zeros(len(pts), dtype=ops.POINT48)
    cloud["x"], cloud["y"], cloud["z"], cloud["w"] = pts[:, 0], pts[:, 1], pts[:, 2], 1.0
    cloud = ops.cloud_to_device(cloud, ctx.device)
    q = torch.from_numpy(np.random.default_rng(1002 + rank).uniform(-10, 10, (100_000, 3))).to(ctx.device)
    n = len(pts)

    def step(timed):
        def run():
            vox = ops.voxel_filter(ctx, cloud, 0.1)
            ix = ops.GridIndex(ctx, vox, stride_bytes=48)
            out = ops.knn(ix, q, 1)
            ix.close()
            return out
        timer(run) if timed else run()

    info = {"unit": "Mpoints/s", "units_per_step": n, "dtype": "f64",
            "workload": "C1: VoxelGrid leaf 0.1f of 105k pts (100k uniform in a 20 m cube + 5% duplicates) "
                        "+ fp64 index + 1-NN of 100k queries",
            "roofline": None}

    def cpu():
        ora = _oracle()
        host = ops.cloud_to_host(cloud)
        qh = q.cpu().numpy()
        def run(th):
            vox, _ = ora.voxel_filter(host, 0.1)
            vx = np.stack([vox["x"], vox["y"], vox["z"]], 1)
            ora.KdTree(vx).knn(qh, 1, nthreads=th)
        dt, th, tried = _fastest(run)
        return {"value": round(n / dt / 1e6, 3), "unit": "Mpoints/s", "cores": th, "kind": "port",
                "sample": f"the whole C1 workload: oracle voxel filter (1 thread) + kd-tree build + 1-NN (OpenMP, "
                          f"the faster of {sorted(tried)} threads: seconds {tried})"}
    return step, info, cpu


def cfg_c2(ctx, args, rank, timer):
    from pointcloudprocess_amd import ops, synth
    n = 1_000_000
    t = synth.uniform_cube(n, 2001 + 1000 * rank, half=50.0, device=ctx.device)
    q = synth.uniform_cube(n, 2002 + 1000 * rank, half=50.0, device=ctx.device)

    def step(timed):
        fn = lambda: ops.knn_bruteforce(ctx, t, q, 8)
        timer(fn) if timed else fn()

    flops = 8.0 * n * n
    info = {"unit": "Mqueries/s", "units_per_step": n, "dtype": "f32",
            "workload": "C2: 1M-vs-1M uniform [-50,50]^3, brute-force kNN k=8 (v_mfma_f32_16x16x4f32 ranking, "
                        "certified fp64 FLANN re-rank)",
            "roofline_fn": lambda ms: {"bound": "mfma", "kernel": "k_bf_mfma (+ re-rank and fallback, one call)",
                                       "achieved": round(flops / ms / 1e9, 2), "peak": F32_MFMA_TFS,
                                       "unit": "TFLOP/s", "frac": round(flops / ms / 1e9 / F32_MFMA_TFS, 4),
                                       "traffic": None, "flops_per_launch": flops, "kernel_avg_ms": round(ms, 4)}}

    def cpu():
        ora = _oracle()
        th = t.cpu().numpy()
        qs = q[:200_000].cpu().numpy()
        t0 = time.perf_counter()
        tree = ora.KdTree(th)
        tb = time.perf_counter() - t0
        dt, th, tried = _fastest(lambda th: tree.knn(qs, 8, nthreads=th))
        return {"value": round(len(qs) / dt / 1e6, 3), "unit": "Mqueries/s", "cores": th, "kind": "port",
                "sample": f"oracle kd-tree (FLANN contract) over the same 1M targets: {len(qs)} queries k=8 in "
                          f"{dt:.2f} s on {th} threads (seconds per thread count {tried}; build {tb:.2f} s, not in "
                          f"value)"}
    return step, info, cpu


def cfg_c3(ctx, args, rank, timer):
    from pointcloudprocess_amd import ops
    n = 10_000_000
    cloud = street_aos48(n, 3001 + 1000 * rank, ctx.device)
    ntimer = Timer()
    state = {}

    def step(timed):
        def run():
            vox = ops.voxel_filter(ctx, cloud, 0.05)
            ix = ops.GridIndex(ctx, vox, stride_bytes=48)
            nrm = ntimer(lambda: ops.normals_knn(ix, 32)) if timed else ops.normals_knn(ix, 32)
            state["m"] = vox.shape[0]
            ix.close()
            return nrm
        timer(run) if timed else run()

    info = {"unit": "Mpoints/s", "units_per_step": n, "dtype": "f64",
            "workload": "C3: 10M-pt street scene (48-B PointXYZRGBA records), VoxelGrid leaf 0.05f, fp64 index of "
                        "the centroids, calculate_feature normals k=32 (FLANN-exact kNN, fp64 PCA)"}

    def roof(ms_step):
        ms = ntimer.avg
        m = state["m"]
        byts = m * (12 + 16)
        return {"bound": "hbm", "kernel": "pcp_normals_knn (k_normals_tile + uncertified-lane passes)",
                "achieved": round(byts / ms / 1e6, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 5), "traffic": None, "kernel_avg_ms": round(ms, 4),
                "units_per_launch": m, "bytes_per_unit": 28,
                "note": "instruction-bound (exact top-32 selection), not memory-bound: 28 B per centroid moves "
                        "in microseconds"}
    info["roofline_fn"] = roof

    def cpu():
        ora = _oracle()
        s = 1_000_000
        host = ops.cloud_to_host(cloud[:s])
        t0 = time.perf_counter()
        vox, _ = ora.voxel_filter(host, 0.05)
        tv = time.perf_counter() - t0
        vx = np.stack([vox["x"], vox["y"], vox["z"]], 1)
        tn, th, tried = _fastest(lambda th: ora.normals_knn(vx, 32, nthreads=th))
        return {"value": round(s / (tv + tn) / 1e6, 3), "unit": "Mpoints/s", "cores": th, "kind": "port",
                "sample": f"the first {s} points: oracle voxel filter {tv:.2f} s (1 thread) + kd-tree normals k=32 "
                          f"over its {len(vx)} centroids {tn:.2f} s (OpenMP on {th} threads; seconds per thread "
                          f"count {tried})"}
    return step, info, cpu


def cfg_c5(ctx, args, rank, timer):
    """N = 1: the 200M-point scene on one GPU.  N > 1 (strong scaling): the SAME scene split into
    equal-count x-slabs, each rank indexing its slab plus the points within r of its faces (the
    halo) and producing the rows and planes of its owned points with global ids; no collective
    (distributed.radius_slab_split_dev)."""
    from pointcloudprocess_amd import distributed as D
    from pointcloudprocess_amd import ops, synth
    world = int(os.environ.get("WORLD_SIZE", "1"))
    R = 0.2
    n = int(args.c5_points)
    side = math.sqrt(n / 1.5e6) * 40.0  # the C5 test density (1.5M pts on 40 x 40 m)
    xyz = synth.street_scene(n, 5001, extent=(side, side), device=ctx.device)
    order = getattr(args, "c5_order", "native")
    if order == "tiles":  # diagnostic: caller order = 1 m tiles, row-major
        t = torch.floor(xyz[:, :2] + side).long()
        xyz = xyz[torch.argsort(t[:, 1] * 100_000 + t[:, 0])].contiguous()
        del t
    elif order == "cells":  # diagnostic: caller order = the index's cell order (z, y, x cells of r)
        c = torch.floor((xyz - xyz.min(0).values) / R).long()
        m = c.max(0).values + 1
        xyz = xyz[torch.argsort((c[:, 2] * m[1] + c[:, 1]) * m[0] + c[:, 0])].contiguous()
        del c
    own = halo = gid = None
    if world > 1:
        own, halo = D.radius_slab_split_dev(xyz[:, 0].contiguous(), world, rank, R)
        gid_t = torch.cat([own, halo])
        xyz = xyz[gid_t].contiguous()
        gid = gid_t.to(torch.int32)
        del gid_t
    n_owned = n if own is None else int(own.numel())
    ktimer = Timer()
    btimer = Timer()
    state = {}

    def step(timed):
        def run():
            ix = btimer(lambda: ops.H16Index(ctx, xyz, cell_size=R)) if timed else ops.H16Index(ctx, xyz, cell_size=R)
            fn = lambda: ix.radius_normals(R, n_owned=n_owned, global_id=gid)
            offs, idx, nrm = ktimer(fn) if timed else fn()
            state["nnz"] = idx.numel()
            ix.close()
            return nrm
        timer(run) if timed else run()

    par = (f"x-slabs x{world}: a rank indexes its equal-count slab + the points within r of its faces "
           f"(halo) and writes its owned points' rows (global ids) and planes; no collective") if world > 1 else \
        "x1"
    info = {"unit": "Mpoints/s", "units_per_step": n_owned, "units_all_ranks_per_step": n,
            "data": "synthetic street scene (seeded)" + ("; one scene split into x-slabs across the ranks"
                                                         if world > 1 else ""),
            "scaling": "strong" if world > 1 else "weak", "parallelism": par,
            "dtype": "fp16 coords / f32 accum",
            "pmc_key": {"n": n, "world": world},
            "workload": f"C5: radiusSearch r=0.2 + normals over the fp16 cell-relative index, the {n}-pt street "
                        f"scene ({side:.0f} x {side:.0f} m)" + (f", split into {world} x-slabs with an r halo"
                                                               if world > 1 else " on one GPU")
                        + ("" if order == "native" else f" [diagnostic: caller order = {order}]")}

    def per_rank():
        return {"owned_points": n_owned, "halo_points": 0 if halo is None else int(halo.numel()),
                "index_build_ms": round(btimer.avg, 3), "rows_normals_ms": round(ktimer.avg, 3)}
    info["per_rank_fn"] = per_rank

    def roof(ms_step):
        ms = ktimer.avg
        nbar = state["nnz"] / max(n_owned, 1)
        byts = n_owned * (6 + 4 * nbar + 16 + 4)
        return {"bound": "hbm", "kernel": "pcp_h16_radius_count + scan + pcp_h16_radius_fill (rows + normals; "
                                          "k_h16_mx on the matrix cores)",
                "achieved": round(byts / ms / 1e6, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(byts / ms / 1e6 / HBM_PEAK_GBS, 4), "traffic": None, "kernel_avg_ms": round(ms, 4),
                "units_per_launch": n_owned, "bytes_per_unit": round(6 + 4 * nbar + 16 + 4, 2), "nbar": round(nbar, 2)}
    info["roofline_fn"] = roof

    def check(nsample=20_000):
        """N > 1: this rank's rows of a seeded global sample of its owned points against the rows of
        the whole cloud indexed on this rank (single-process rows): equal as sets except pairs
        within the fp16 band of r (the slab's grid origin quantises differently)."""
        full = synth.street_scene(n, 5001, extent=(side, side), device=ctx.device)
        ixf = ops.H16Index(ctx, full, cell_size=R)
        offs_f, idx_f, _ = ixf.radius_normals(R, normals=False)
        ixf.close()
        ix = ops.H16Index(ctx, xyz, cell_size=R)
        offs_l, idx_l, _ = ix.radius_normals(R, n_owned=n_owned, global_id=gid, normals=False)
        ix.close()
        g = torch.Generator(device="cpu")
        g.manual_seed(77 + rank)
        pick = torch.randint(0, n_owned, (nsample,), generator=g).to(ctx.device)
        gq = own[pick]

        def pairs(offs, idx, s):  # (sample slot * n + neighbour id) of the rows of queries s
            lens = offs[s + 1] - offs[s]
            row_of = torch.repeat_interleave(torch.arange(s.numel(), device=s.device), lens)
            pos = offs[s][row_of] + (torch.arange(row_of.numel(), device=s.device) - (torch.cumsum(lens, 0) - lens)[row_of])
            return row_of * n + idx[pos].long()
        keys, cnt = torch.unique(torch.cat([pairs(offs_l, idx_l, pick), pairs(offs_f, idx_f, gq)]), return_counts=True)
        odd = keys[cnt == 1]  # in one of the two rows only
        d = torch.linalg.norm(full[odd % n].double() - full[gq[odd // n]].double(), dim=1)
        diff_out = int(odd.numel())
        bad = int(((d - R).abs() >= 3e-4).sum())
        return {"sampled_rows": nsample, "pairs_differing": diff_out, "pairs_differing_outside_band": bad}
    info["check_fn"] = check

    def cpu():
        ora = _oracle()
        ns, s = 2_000_000, 500_000
        side_s = math.sqrt(ns / 1.5e6) * 40.0  # a tile of the same scene at the same density
        xh = synth.street_scene(ns, 5001, extent=(side_s, side_s), device="cpu").numpy().astype(np.float64)
        t0 = time.perf_counter()
        tree = ora.KdTree(xh)
        tb = time.perf_counter() - t0
        qs = np.sort(np.random.default_rng(5).choice(ns, s, replace=False)).astype(np.int32)
        res = {}
        dt, th, tried = _fastest(lambda th: res.update(c=tree.radius_normals(qs, 0.2, nthreads=th)[0]))
        cnt = res["c"]
        return {"value": round(s / dt / 1e6, 4), "unit": "Mpoints/s", "cores": th, "kind": "port",
                "sample": f"{s} random points of a {ns}-pt tile of the same scene at the same density "
                          f"({side_s:.0f} x {side_s:.0f} m): oracle kd-tree radiusSearch r=0.2 (sorted rows) + fp64 F1 "
                          f"per point, OpenMP over points (ora_radius_normals_batch) on {th} threads (seconds per "
                          f"thread count {tried}), nbar {cnt.mean():.1f}, in {dt:.2f} s; kd-tree build {tb:.1f} s "
                          f"not in value"}
    return step, info, cpu


def main(args):
    import torch.distributed as dist
    from pointcloudprocess_amd import ops
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = int(os.environ.get("PCP_BENCH_DEVICE", local))  # rehearsal: every rank on one device
    backend = os.environ.get("PCP_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    ctx = ops.Context(local)

    def barrier():
        if world > 1:
            dist.barrier()

    def reduce(x, op):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    timer = Timer()
    step, info, cpu = {"C1": cfg_c1, "C2": cfg_c2, "C3": cfg_c3, "C5": cfg_c5}[args.config](ctx, args, rank, timer)
    dt = run_steps(step, args.steps, args.warmup, barrier)
    dt = reduce(dt, dist.ReduceOp.MAX if world > 1 else None)
    units = info.get("units_all_ranks_per_step", info["units_per_step"] * world) * args.steps
    per_rank = None
    if "per_rank_fn" in info and world > 1:
        mine = info["per_rank_fn"]()
        keys = sorted(mine)
        slots = torch.zeros(world * len(keys), dtype=torch.float64, device=dev)
        for j, k in enumerate(keys):
            slots[rank * len(keys) + j] = float(mine[k])
        dist.all_reduce(slots, op=dist.ReduceOp.SUM)
        slots = slots.cpu().tolist()
        per_rank = [{"rank": r, **{k: slots[r * len(keys) + j] for j, k in enumerate(keys)}} for r in range(world)]
    check = None
    if getattr(args, "c5_check", 0) and "check_fn" in info and world > 1:
        mine = info["check_fn"](args.c5_check)
        t = torch.tensor([float(mine[k]) for k in sorted(mine)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        check = {k: int(v) for k, v in zip(sorted(mine), t.cpu().tolist())}
    roof = info.get("roofline_fn")
    line = {
        "metric": f"{args.config} throughput ({info['unit']})",
        "value": round(units / dt / 1e6, 3),
        "unit": info["unit"],
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": info.get("scaling", "weak"),
        "vs_baseline": None,
        "dtype": info["dtype"],
        "data": info.get("data", "synthetic (seeded)" + ("; every rank its own batch" if world > 1 else "")),
        "config": {"workload": info["workload"],
                   "parallelism": info.get("parallelism", f"x{world} independent batches, no collective")},
        "per_rank": per_rank,
        "slab_rows_check": check,
        "device_ms_per_step": round(timer.avg, 3),
        "roofline": _with_traffic(roof(timer.avg), args.config, info.get("pmc_key", {"n": info["units_per_step"],
                                                                                     "world": world})) if roof else None,
        "build_id": ctx.lib.pcp_build_id().decode(),  # SHA-1 of the libpcp sources (provenance)
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = _cpu_meta(cpu())
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return 0
