"""Multi-GPU drivers of the ICP correspondence/transform loop.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on the MI355X node,
"gloo" in the CPU tests).  The loop body is the same on every rank; only the reduction
differs between the two partitionings:

* co-partitioned (bench.py default): each rank owns a spatial tile of BOTH clouds (query
  tile + target tile widened by a halo >= the largest correspondence distance), so every
  correspondence is found locally; the only collective is all_reduce(SUM) of the 24 fp64
  accumulators per iteration (192 bytes).
* target-sharded (the north_star layout): each rank indexes one shard of the target, the
  query set is replicated.  Per iteration: per-query int64 keys (fp32 d2 bits << 32 |
  global target index) -> all_reduce(MIN) gives the global lexicographic (d2, index)
  winner; each rank accumulates the queries whose winner lies in its shard ->
  all_reduce(SUM) of the 24 accumulators.  8 bytes per query per iteration cross xGMI, so
  it scales worse than co-partitioning; it needs no spatial partition of the queries.

An *engine* supplies the local compute:
    step(T, rmax) -> acc            (24 float64, torch tensor on the engine's device)
    keys(T, rmax, offset) -> keys   (int64 torch tensor, one per query)
    accumulate_keys(T, keys, lo, hi) -> acc
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


def shard_range(n, world, rank):
    """Equal-count contiguous shard [lo, hi) of n items."""
    lo = (n * rank) // world
    return lo, (n * (rank + 1)) // world


class GpuEngine:
    """libpcp engine: fp32 grid index over the local target (tile or shard) + the queries."""

    def __init__(self, ctx, target_xyz, query_xyz, cell_size=0.0):
        self.target = target_xyz.contiguous()
        self.index = ops.GridIndex(ctx, self.target, cell_size=cell_size)
        self.icp = ops.ICP(self.index, query_xyz.contiguous())

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

    def close(self):
        self.icp.close()
        self.index.close()
