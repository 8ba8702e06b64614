"""Multi-GPU drivers of the ICP correspondence/transform loop.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on the MI355X node,
"gloo" in the CPU tests).  The loop body is the same on every rank; only the reduction
differs between the two partitionings:

* co-partitioned (bench.py default): each rank owns a spatial tile of BOTH clouds (query
  tile + target tile widened by a halo >= the largest correspondence distance), so every
  correspondence is found locally; the only collective is all_reduce(SUM) of the 24 fp64
  accumulators per iteration (192 bytes).
* slab (bench.py headline, strong scaling): ONE registration split by x-slabs -- a rank owns
  the queries of its slab and indexes the targets of the slab widened by a halo; a device
  guard certifies every iteration that the pose keeps the owned queries inside the halo.
  Collective: all_reduce(SUM) of 24 doubles per iteration.
* target-sharded (the north_star layout): each rank indexes one shard of the target, the
  query set is replicated.  Per iteration: per-query int64 keys (fp32 d2 bits << 32 |
  global target index) -> MIN over ranks gives the global lexicographic (d2, index)
  winner (all_reduce + per-shard accumulation, or -- device-resident -- ReduceScatter(MIN),
  an AllGather of the winners' owning shard (1 byte per query) and accumulation of the owned
  winners from the rank's own shard) -> all_reduce(SUM) of the 24 accumulators.  No rank holds
  more than its shard of the target; 8 + 1 bytes per query per iteration cross xGMI, so it
  scales worse than co-partitioning; it needs no spatial partition of the queries.

An *engine* supplies the local compute:
    step(T, rmax) -> acc            (24 float64, torch tensor on the engine's device)
    keys(T, rmax, offset) -> keys   (int64 torch tensor, one per query)
    accumulate_keys(T, keys, lo, hi) -> acc
    keys_dev(T_dev, rmax, offset, out), key_owner(keys, bounds, out),
    accumulate_owned(T_dev, keys, owner, rank, lo, hi) -> acc   (device-resident sharded loop)
and, for the device-resident loop (run_copartitioned_dev: the pose and the solve stay on
the device, the all-reduce is enqueued on the same stream, no host round trip per
iteration):
    new_pose(T0) -> (T_dev, stats)  (16 + 4 float64 tensors on the engine's device)
    step_dev(T_dev, rmax) -> acc
    solve_dev(acc, T_dev, stats, do_scale)
GpuEngine is the libpcp implementation; tests/oracle_engine.py restates it on the CPU.
"""
import math

import numpy as np
import torch
import torch.distributed as dist

from . import ops


def _world():
    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


def _allreduce(t, op):
    if _world() > 1:
        if t.is_cuda and dist.get_backend() == "gloo":  # (one-GPU rehearsals: through host memory)
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)
    return t


def _finish(acc_t, T, do_scale):
    a = acc_t.detach().cpu().numpy()
    rc, dT = ops.icp_solve(a, do_scale)
    if rc != 0:
        return None, -1.0
    return dT @ T, math.sqrt(a[22] / a[0])


def run_copartitioned(engine, T0, rmax, iters, do_scale=False):
    """ICP over co-partitioned tiles; returns (err, T) -- identical on every rank."""
    T = np.array(T0, dtype=np.float64)
    err = -1.0
    for _ in range(iters):
        acc = _allreduce(engine.step(T, rmax).clone(), dist.ReduceOp.SUM)
        Tn, err = _finish(acc, T, do_scale)
        if Tn is None:
            return -1.0, T
        T = Tn
    return err, T


def run_copartitioned_dev(engine, T0, rmax, iters, do_scale=False):
    """run_copartitioned with the pose, solve and all-reduce kept on the device stream (the
    bench's loop); one host sync at the end.  Returns (err, T) -- identical on every rank."""
    T_dev, stats = engine.new_pose(T0)
    for _ in range(iters):
        acc = engine.step_dev(T_dev, rmax)
        _allreduce(acc, dist.ReduceOp.SUM)
        engine.solve_dev(acc, T_dev, stats, do_scale)
    st = stats.cpu().numpy()
    T = T_dev.cpu().numpy().reshape(4, 4)
    return (float(st[1]) if st[0] == 0 and st[3] == iters else -1.0), T


def run_target_sharded(engine, T0, rmax, iters, lo, hi, do_scale=False):
    """ICP with the target sharded over ranks ([lo, hi) = this rank's global target range)."""
    T = np.array(T0, dtype=np.float64)
    err = -1.0
    for _ in range(iters):
        keys = _allreduce(engine.keys(T, rmax, lo), dist.ReduceOp.MIN)
        acc = _allreduce(engine.accumulate_keys(T, keys, lo, hi).clone(), dist.ReduceOp.SUM)
        Tn, err = _finish(acc, T, do_scale)
        if Tn is None:
            return -1.0, T
        T = Tn
    return err, T


NO_KEY = torch.iinfo(torch.int64).max


def _reduce_scatter_min(out, inp):
    """out <- this rank's equal slice of the element-wise MIN over ranks of inp (RCCL
    ReduceScatter; gloo, which has none, reduces everything and keeps the slice)."""
    world = _world()
    if world == 1:
        out.copy_(inp)
    elif dist.get_backend() == "gloo":  # (rehearsals on one GPU / CPU tests: through host memory)
        h = inp.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MIN)
        out.copy_(h.view(world, -1)[dist.get_rank()])
    else:
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.MIN)
    return out


def _all_gather_bytes(out, inp):
    """out <- the concatenation over ranks of inp (equal-size slices)."""
    world = _world()
    if world == 1:
        out.copy_(inp)
    elif dist.get_backend() == "gloo":  # (rehearsals on one GPU / CPU tests: through host memory)
        parts = [torch.empty_like(inp, device="cpu") for _ in range(world)]
        dist.all_gather(parts, inp.cpu())
        out.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(out, inp)
    return out


def run_target_sharded_dev(engine, T0, rmax, iters, bounds, do_scale=False, exchange=None):
    """The north_star layout with the pose on the device and no rank holding more of the target
    than its own shard.  Every rank indexes its shard (global target indices [bounds[r],
    bounds[r + 1])) and holds the replicated queries.  Per iteration (no host round trip):
      keys at the device pose (this rank's local winners, 8 B per query)
      -> ReduceScatter(MIN): the global winners of this rank's 1/G slice of the queries
      -> the owning shard of each of those winners (1 B per query) -> AllGather
      -> accumulators of the queries whose winner this rank owns, read from its own shard
      -> all_reduce(SUM) of 24 doubles -> device solve.
    `exchange`: optional list that receives (start, end) CUDA event pairs around the two
    per-query collectives of each iteration.  Returns (err, T), identical on every rank."""
    world = _world()
    rank = dist.get_rank() if world > 1 else 0
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    nq = engine.nq
    dev = engine.device
    chunk = -(-nq // world)
    keys = torch.full((chunk * world,), NO_KEY, dtype=torch.int64, device=dev)
    mine = torch.empty(chunk, dtype=torch.int64, device=dev)
    own_mine = torch.empty(chunk, dtype=torch.uint8, device=dev)
    owner = torch.empty(chunk * world, dtype=torch.uint8, device=dev)
    bnd = torch.tensor([int(b) for b in bounds], dtype=torch.int64, device=dev)
    T_dev, stats = engine.new_pose(T0)
    for _ in range(iters):
        engine.keys_dev(T_dev, rmax, lo, keys)
        ev = None
        if exchange is not None and keys.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        _reduce_scatter_min(mine, keys.clone() if keys.device.type == "cpu" else keys)  # (gloo reduces in place)
        engine.key_owner(mine, bnd, own_mine)
        _all_gather_bytes(owner, own_mine)
        if ev is not None:
            ev[1].record()
            exchange.append(ev)
        acc = engine.accumulate_owned(T_dev, keys, owner, rank, lo, hi)
        _allreduce(acc, dist.ReduceOp.SUM)
        engine.solve_dev(acc, T_dev, stats, do_scale)
    st = stats.cpu().numpy()
    T = T_dev.cpu().numpy().reshape(4, 4)
    return (float(st[1]) if st[0] == 0 and st[3] == iters else -1.0), T


def slab_bounds(x, world):
    """x-slab boundaries (world + 1 values, -inf/+inf at the ends) cutting the values x into
    equal-count slabs (the same on every rank for the same x)."""
    xs = np.sort(np.asarray(x, dtype=np.float64))
    b = [-np.inf]
    for r in range(1, world):
        b.append(float(xs[(len(xs) * r) // world]) if len(xs) else 0.0)
    b.append(np.inf)
    return b


def slab_select(q_x, t_x, bounds, rank, halo):
    """Masks of this rank's owned queries (x in [b_r, b_r+1)) and target tile (the slab
    widened by `halo` on both sides)."""
    lo, hi = bounds[rank], bounds[rank + 1]
    return (q_x >= lo) & (q_x < hi), (t_x >= lo - halo) & (t_x < hi + halo)


def run_slab_dev(engine, T0, rmax, iters, guard=None, do_scale=False, exchange=None, out_stats=None):
    """Co-partitioned strong scaling of ONE registration: every rank owns an x-slab of the
    queries and indexes the targets of that slab widened by a halo, so every correspondence
    is found locally; the only collective is all_reduce(SUM) of the 24 accumulators per
    iteration, on the device stream.  guard = (box, lo, hi): the owned queries' box and the x
    range over which the halo certifies them; a device flag latches if the pose ever takes
    the box outside (the result is then not certified).  Returns (err, T, guard_ok)."""
    T_dev, stats = engine.new_pose(T0)
    flag = torch.zeros(1, dtype=torch.int32, device=T_dev.device)
    for _ in range(iters):
        if guard is not None:
            engine.slab_guard(T_dev, guard[0], guard[1], guard[2], flag)
        acc = engine.step_dev(T_dev, rmax)
        ev = None
        if exchange is not None and T_dev.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        _allreduce(acc, dist.ReduceOp.SUM)
        if ev is not None:
            ev[1].record()
            exchange.append(ev)
        engine.solve_dev(acc, T_dev, stats, do_scale)
    # one device->host copy (and one sync) for the stats, the pose and the guard flag
    ns = stats.numel()
    host = torch.cat([stats.reshape(-1).double(), T_dev.reshape(-1).double(), flag.double()]).cpu().numpy()
    st, T, ok = host[:ns], host[ns:ns + 16].reshape(4, 4).copy(), bool(host[ns + 16] == 0)
    if out_stats is not None:
        out_stats["fallback"] = float(st[2])  # queries that needed the exact fallback, all iterations
    return (float(st[1]) if st[0] == 0 and st[3] == iters else -1.0), T, ok


def shard_range(n, world, rank):
    """Equal-count contiguous shard [lo, hi) of n items."""
    lo = (n * rank) // world
    return lo, (n * (rank + 1)) // world


class GpuEngine:
    """libpcp engine: fp32 grid index over the local target (tile or shard) + the queries."""

    # profiling only (bench.py --oct-lanes-list ...): (oct_lanes_first, oct_lanes_list, ring_lanes)
    # passed to ICP.set_options on every new handle; None = the library's own choices
    lane_options = None
    graph = False  # bench.py --icp-graph: PCP_ICP_OPT_GRAPH on every new handle

    def __init__(self, ctx, target_xyz, query_xyz, cell_size=0.0):
        self.target = target_xyz.contiguous()
        # the index build and the query sort in one call (their radix sorts overlap on two streams)
        if hasattr(ctx.lib, "pcp_icp_create_with_target"):
            self.icp = ops.ICP.with_target(ctx, self.target, query_xyz.contiguous(), cell_size)
            self.index = self.icp.index
        else:  # (an A/B build of an older tree, PCP_LIB)
            self.index = ops.GridIndex(ctx, self.target, cell_size=cell_size)
            self.icp = ops.ICP(self.index, query_xyz.contiguous())
        if GpuEngine.lane_options is not None or GpuEngine.graph:
            self.icp.set_options(*(GpuEngine.lane_options or (1, 0, 0)), graph=GpuEngine.graph)
        self.device = ctx.device
        self.nq = query_xyz.shape[0]

    def step(self, T, rmax):
        return self.icp.step(T, rmax)

    def keys(self, T, rmax, offset):
        return self.icp.keys(T, rmax, offset)

    def new_pose(self, T0):
        return self.icp.new_pose(T0)

    def step_dev(self, T_dev, rmax):
        return self.icp.step_dev(T_dev, rmax)

    def solve_dev(self, acc, T_dev, stats, do_scale=False):
        self.icp.solve_dev(acc, T_dev, stats, do_scale)

    def accumulate_keys(self, T, keys, lo, hi):
        return self.icp.accumulate_keys(T, keys, lo, hi, self.target)

    def keys_dev(self, T_dev, rmax, offset, out=None):
        return self.icp.keys_dev(T_dev, rmax, offset, out)

    def key_owner(self, keys, bounds, out):
        return ops.keys_owner(self.index.ctx, keys, bounds, out)

    def accumulate_owned(self, T_dev, keys, owner, rank, lo, hi):
        return ops.accumulate_owned(self.index.ctx, T_dev, self.icp.q, keys, owner, rank, lo, hi, self.target,
                                    self.icp.acc)

    def slab_guard(self, T_dev, box, lo, hi, flag):
        ops.slab_guard(self.index.ctx, T_dev, box, lo, hi, flag)

    def close(self):
        self.icp.close()
        self.index.close()


# ---- C5 radius + normals over x-slabs with an r-wide halo ("for radius,
# exchange a halo of width r between slabs instead, so no per-query collective is needed")
def radius_slab_split(x, world, rank, r):
    """(owned, halo) indices of this rank's x-slab of the points with x-coordinates `x`:
    equal-count slabs, halo = the points within r of the slab's faces (on the neighbours)."""
    b = slab_bounds(x, world)
    lo, hi = b[rank], b[rank + 1]
    x = np.asarray(x)
    own = np.nonzero((x >= lo) & (x < hi))[0]
    halo = np.nonzero(((x >= lo - r) & (x < lo)) | ((x >= hi) & (x < hi + r)))[0]
    return own, halo


def radius_slab_split_dev(x, world, rank, r):
    """radius_slab_split on a device tensor of x-coordinates (the C5 bench's 200M-point cloud
    stays in HBM): the same equal-count bounds (sorted x at n * k / world, as slab_bounds, in the
    values' own precision) and the same owned / halo sets, as int64 index tensors in ascending
    order."""
    n = x.numel()
    xs = torch.sort(x.double()).values
    b = [-math.inf] + [float(xs[(n * k) // world]) if n else 0.0 for k in range(1, world)] + [math.inf]
    del xs
    lo, hi = b[rank], b[rank + 1]
    xd = x.double()
    own = torch.nonzero((xd >= lo) & (xd < hi)).flatten()
    halo = torch.nonzero(((xd >= lo - r) & (xd < lo)) | ((xd >= hi) & (xd < hi + r))).flatten()
    return own, halo


def radius_rows_slab(engine, xyz, r, world=None, rank=None):
    """Rows (CSR over this rank's owned points, global ids) of the radius search with the
    slab split; engine.radius_rows(local_xyz, n_owned, gid, r) -> (offsets, idx) does the
    local search over owned + halo points.  No collective: every row is complete locally."""
    world = _world() if world is None else world
    rank = (dist.get_rank() if world > 1 else 0) if rank is None else rank
    own, halo = radius_slab_split(np.asarray(xyz)[:, 0], world, rank, r)
    gid = np.concatenate([own, halo]).astype(np.int32)
    offs, idx = engine.radius_rows(np.asarray(xyz)[gid], len(own), gid, r)
    return own, offs, idx
