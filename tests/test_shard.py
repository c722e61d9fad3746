"""CPU: multi-GPU sharding logic on gloo, world_size 2.

The per-rank solver is injected; here it is the CPU oracle (test infrastructure),
so the check is purely that partition + gather reproduce the unsharded batch in
global order.  The GPU solver behind the same partition is covered by
tests/test_gpu_parity.py::test_sharded_solve_matches_unsharded."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from trajectory_generator_ros2_amd import METHOD_DENSE_KKT, METHOD_REDUCED
from trajectory_generator_ros2_amd import shard as SH
from trajectory_generator_ros2_amd import synthetic as S


def test_uniform_bounds():
    np.testing.assert_array_equal(SH.uniform_bounds(10, 4), [0, 3, 6, 8, 10])
    np.testing.assert_array_equal(SH.uniform_bounds(0, 2), [0, 0, 0])
    np.testing.assert_array_equal(SH.uniform_bounds(65536 * 8, 8), np.arange(9) * 65536)


@pytest.mark.parametrize("method", [METHOD_REDUCED, METHOD_DENSE_KKT])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_ragged_bounds_balanced_and_contiguous(method, world):
    so, _, _ = S.ragged_batch(5000, 2, 16)
    b = SH.ragged_bounds(so, world, method)
    assert b[0] == 0 and b[-1] == 5000 and (np.diff(b) >= 0).all()
    cost = SH.trajectory_cost(np.diff(so), method)
    per = np.add.reduceat(cost, b[:-1][np.diff(b) > 0]) if world > 1 else np.array([cost.sum()])
    assert per.max() <= cost.sum() / world + cost.max() + 1e-6


def test_ragged_bounds_more_ranks_than_trajectories():
    so = np.array([0, 3, 5], dtype=np.int32)
    b = SH.ragged_bounds(so, 4)
    assert b[0] == 0 and b[-1] == 2 and (np.diff(b) >= 0).all()


def test_shard_csr_slices():
    so, W, T = S.ragged_batch(50, 2, 6)
    Wf, Tf = W.reshape(-1, 3), T.reshape(-1)
    so_l, W_l, T_l, ED_l = SH.shard_csr(so, Wf, Tf, None, 10, 20)
    assert so_l[0] == 0 and so_l.shape == (11,)
    assert W_l.shape[0] == int(so_l[-1]) + 10 and T_l.shape[0] == int(so_l[-1])
    np.testing.assert_array_equal(W_l[0], Wf[so[10] + 10])
    np.testing.assert_array_equal(T_l, Tf[so[10]:so[20]])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ragged, q):
    import torch.distributed as dist

    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if ragged:
            so, W, T = S.ragged_batch(301, 1, 16, seed=7)
        else:
            so, W, T = S.uniform_batch(301, 10, seed=7)
        sb = SH.ShardedBatch(so, W.reshape(-1, 3), T.reshape(-1), None, rank=rank, world=world)
        C, st = sb.solve(lambda so_, W_, T_, ED_: O.solve_batch(so_, W_, T_, ED_, O.KKT_C4, 1))
        out = sb.gather(C, st, dst=0)
        if rank == 0:
            Cf, stf = O.solve_batch(so, W.reshape(-1, 3), T.reshape(-1), None, O.KKT_C4, 1)
            ok = out[0].shape == Cf.shape and np.array_equal(out[0].numpy(), Cf) and \
                np.array_equal(out[1].numpy(), stf)
            q.put(bool(ok))
        else:
            q.put(out is None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ragged", [False, True])
def test_gloo_world2_shard_and_gather(ragged, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ragged, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = [q.get(timeout=5) for _ in range(2)]
    assert all(res)


def _pipelined_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, M = 203, 4
        so, W, T = S.uniform_batch(B, M, seed=S.SEED + rank)
        C = torch.zeros((B, M, 3, 8), dtype=torch.float64)

        def solve_chunk(lo, hi):
            c, st = O.solve_batch(so[lo:hi + 1] - so[lo], W[lo:hi].reshape(-1, 3), T[lo:hi].reshape(-1), None,
                                  O.KKT_C4, 1)
            assert (st == 0).all()
            C[lo:hi] = torch.from_numpy(c.reshape(hi - lo, M, 3, 8))

        out = torch.full((world, B, M, 3, 8), float("nan"), dtype=torch.float64) if rank == 0 else None
        for w in SH.pipelined_gather(solve_chunk, C, chunks=5, dst=0, out=out):
            w.wait()
        if rank == 0:
            ok = True
            for r in range(world):
                so_r, W_r, T_r = S.uniform_batch(B, M, seed=S.SEED + r)
                ref, _ = O.solve_batch(so_r, W_r.reshape(-1, 3), T_r.reshape(-1), None, O.KKT_C4, 1)
                ok &= np.array_equal(out[r].numpy().reshape(-1, 3, 8), ref)
            q.put(bool(ok))
        else:
            q.put(True)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_pipelined_gather(oracle):
    """bench.py's config-4 line: chunked solve + per-chunk gather to rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert all(q.get(timeout=5) for _ in range(2))
