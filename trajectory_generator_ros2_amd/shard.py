"""Multi-GPU sharding of a trajectory batch.

Trajectories are independent, so the solve shards with no collective on the data
path: one process per GPU (torch.distributed, RCCL backend "nccl" on MI355X), each
solving a contiguous trajectory range on its own device.  The only exchange is the
optional final coefficient gather to one rank (§8(e) "one final coefficient gather"),
used when a caller wants every trajectory in one place; the benchmark does not.

Partitioning:
  uniform batches   equal contiguous ranges (remainder spread over the first ranks)
  ragged batches    contiguous ranges balanced by the prefix sum of the kernel's cost
                    per trajectory (§8(e)): reduced method ~ M_b (bytes and flops are
                    both linear in M), dense KKT ~ (14 M_b + 2)^3
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from ._lib import METHOD_DENSE_KKT, METHOD_REDUCED


def uniform_bounds(B: int, world: int) -> np.ndarray:
    """[world+1] trajectory boundaries of equal contiguous shards."""
    if B < 0 or world < 1:
        raise ValueError("B >= 0 and world >= 1 required")
    q, r = divmod(B, world)
    sizes = np.full(world, q, dtype=np.int64)
    sizes[:r] += 1
    return np.concatenate([[0], np.cumsum(sizes)])


def trajectory_cost(seg_counts: np.ndarray, method: int = METHOD_REDUCED) -> np.ndarray:
    m = np.asarray(seg_counts, dtype=np.float64)
    if method == METHOD_DENSE_KKT:
        return (14.0 * m + 2.0) ** 3
    return 2.0 + m  # per-trajectory fixed part (setup, interface solve) + per-segment part


def ragged_bounds(seg_offsets, world: int, method: int = METHOD_REDUCED) -> np.ndarray:
    """[world+1] contiguous trajectory boundaries with ~equal cost per shard."""
    so = np.asarray(seg_offsets, dtype=np.int64)
    B = so.shape[0] - 1
    if world < 1:
        raise ValueError("world >= 1 required")
    if B == 0:
        return np.zeros(world + 1, dtype=np.int64)
    c = np.cumsum(trajectory_cost(np.diff(so), method))
    targets = c[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(c, targets, side="left") + 1
    cuts = np.minimum(np.maximum.accumulate(cuts), B)
    return np.concatenate([[0], cuts, [B]]).astype(np.int64)


def shard_csr(seg_offsets, waypoints, seg_times, end_derivs, lo: int, hi: int):
    """Slice trajectories [lo, hi) out of a CSR batch (include/tgms.h layout); the
    returned seg_offsets start at 0."""
    so = np.asarray(seg_offsets, dtype=np.int64)
    W = np.asarray(waypoints).reshape(-1, 3)
    T = np.asarray(seg_times).reshape(-1)
    s0, s1 = int(so[lo]), int(so[hi])
    so_l = (so[lo:hi + 1] - s0).astype(np.int32)
    W_l = W[s0 + lo:s1 + hi]
    T_l = T[s0:s1]
    ED_l = None if end_derivs is None else np.asarray(end_derivs).reshape(-1, 18)[lo:hi]
    return so_l, W_l, T_l, ED_l


class ShardedBatch:
    """This rank's share of a global CSR batch and the gather of the results.

    solve_fn(so, W, T, ED) -> (coeffs [S,3,8], status [B]) is the per-rank solver: the
    GPU solver (solver.Solver.solve) in production; tests pass other callables to
    check the partition/gather logic on CPU ranks.
    """

    def __init__(self, seg_offsets, waypoints, seg_times, end_derivs=None, *, rank: int = 0, world: int = 1,
                 method: int = METHOD_REDUCED):
        self.so = np.asarray(seg_offsets, dtype=np.int64)
        self.rank, self.world = rank, world
        self.bounds = ragged_bounds(self.so, world, method)
        lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.lo, self.hi = lo, hi
        self.local = shard_csr(self.so, waypoints, seg_times, end_derivs, lo, hi)

    def solve(self, solve_fn: Callable):
        so, W, T, ED = self.local
        return solve_fn(so, W, T, ED)

    def gather(self, coeffs, status, dst: int = 0, group=None) -> Optional[tuple]:
        """Collect every rank's (coeffs, status) on rank `dst` in global trajectory
        order; returns None on the other ranks.  One padded torch.distributed.gather per
        array (equal sizes, as ncclGather requires) — the only collective of the path."""
        import torch
        import torch.distributed as dist

        dev = coeffs.device if isinstance(coeffs, torch.Tensor) else torch.device("cpu")
        C = torch.as_tensor(coeffs, device=dev).reshape(-1, 24)
        St = torch.as_tensor(status, device=dev).reshape(-1)
        seg_per_rank = np.diff(self.so[self.bounds])
        traj_per_rank = np.diff(self.bounds)
        smax, tmax = int(max(seg_per_rank.max(), 1)), int(max(traj_per_rank.max(), 1))
        Cp = torch.zeros((smax, 24), dtype=C.dtype, device=dev)
        Cp[: C.shape[0]] = C
        Sp = torch.zeros((tmax,), dtype=St.dtype, device=dev)
        Sp[: St.shape[0]] = St
        if self.world == 1:
            return C.reshape(-1, 3, 8), St
        me = dist.get_rank(group)
        cl = [torch.empty_like(Cp) for _ in range(self.world)] if me == dst else None
        sl = [torch.empty_like(Sp) for _ in range(self.world)] if me == dst else None
        # `dst` is a rank of `group` (group_dst), compared with the group-local rank above
        dist.gather(Cp, cl, group=group, group_dst=dst)
        dist.gather(Sp, sl, group=group, group_dst=dst)
        if me != dst:
            return None
        Call = torch.cat([cl[r][: int(seg_per_rank[r])] for r in range(self.world)])
        Sall = torch.cat([sl[r][: int(traj_per_rank[r])] for r in range(self.world)])
        return Call.reshape(-1, 3, 8), Sall


def pipelined_gather(solve_chunk: Callable, coeffs, chunks: int, dst: int = 0, out=None, group=None):
    """Solve this rank's uniform shard in `chunks` pieces and gather every piece to
    rank `dst` while the next one is being solved (the final
    coefficient gather, overlapped with the compute in chunks).

    coeffs   this rank's [B, ...] coefficient tensor (every rank the same B)
    solve_chunk(lo, hi)  enqueues the solve of trajectories [lo, hi) into coeffs[lo:hi]
             on the current stream (GPU) or computes it (CPU tests)
    out      on rank dst: a [world, B, ...] tensor that receives every rank's shard in
             rank order (rank-major = global trajectory order for contiguous shards);
             ignored elsewhere

    Each piece is one torch.distributed.gather (ncclSend/ncclRecv under RCCL, issued
    on the communicator's stream after the piece's solve), so the transfer of piece
    c runs beside the solve of piece c + 1.  Returns the list of async works (the
    caller waits on them)."""
    import torch.distributed as dist

    B = coeffs.shape[0]
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    bounds = uniform_bounds(B, max(1, chunks))
    works = []
    for c in range(len(bounds) - 1):
        lo, hi = int(bounds[c]), int(bounds[c + 1])
        if hi <= lo:
            continue
        solve_chunk(lo, hi)
        gl = [out[r, lo:hi] for r in range(world)] if me == dst else None
        works.append(dist.gather(coeffs[lo:hi], gl, group=group, group_dst=dst, async_op=True))
    return works
