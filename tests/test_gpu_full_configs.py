"""BASELINE configs 4 and 5 at their stated size: 1,048,576 trajectories per call,
through the shipped multi-GPU C ABI (tgms_create_multi + tgms_solve_batch_multi_device
/ tgms_refine_loop_multi_device, include/tgms.h) on one MI355X (device_count = 1).

Two modes of the same handle type:
  in_place          device 0's shard (here: the whole batch) is solved in place on the
                    caller's stream;
  rccl_self_gather  TGMS_MULTI_SELF_GATHER=1 routes it through the RCCL pipeline the
                    8-GPU split uses: the batch is cut into cost-balanced pieces
                    (tgms_plan_shards), every piece's inputs are scattered into the
                    device workspace, solved there and gathered back with grouped
                    ncclSend / ncclRecv -- ~2 GB of coefficients at config 4.

Checks: every status OK; the oracle on 1,024-trajectory slices at
the start, the end and across every piece boundary (norm-wise 1e-9 per trajectory
and axis for a solve); the min-snap spline properties on EVERY trajectory
(conftest.check_spline_properties_torch: interpolation, C1..C6 continuity, rest
ends); and bit equality with the single-device entry point on the same batch.
Config 5's refinement: times and costs after 10 steps against the oracle's restatement
of the step at 1e-9 (test_gpu_configs.py's docstring: round 5 needed 1e-7 while the
oracle's gradient was ~1e-8 off exact), the final solve at the GPU's final times to 1e-9.
"""
import os

import numpy as np
import pytest

from conftest import batch_rel_err, check_spline_properties_torch

pytestmark = pytest.mark.gpu

TOL = 1e-9
REFINE_TOL_MAX = 1e-9
B_FULL = 1048576


@pytest.fixture(params=[False, True], ids=["in_place", "rccl_self_gather"])
def multi(request):
    from trajectory_generator_ros2_amd.solver import Solver
    old = os.environ.pop("TGMS_MULTI_SELF_GATHER", None)
    if request.param:
        os.environ["TGMS_MULTI_SELF_GATHER"] = "1"  # read by tgms_create_multi
    try:
        s = Solver(device_count=1)
    finally:
        os.environ.pop("TGMS_MULTI_SELF_GATHER", None)
        if old is not None:
            os.environ["TGMS_MULTI_SELF_GATHER"] = old
    s.self_gather = request.param
    yield s
    s.close()


def _slices(so, n=1024):
    """First, last, and one straddling every boundary of the 4 pieces the multi
    pipeline cuts a one-device shard into (tgms_plan_shards, the library's own rule)."""
    from trajectory_generator_ros2_amd.solver import plan_shards
    B = len(so) - 1
    cuts = [int(c) for c in plan_shards(so, 4)[1:-1]]
    out = [(0, n), (B - n, B)] + [(max(0, c - n // 2), min(B, c + n // 2)) for c in cuts]
    assert len(out) >= 4
    return out


def test_config4_full_size(solver, oracle, multi):
    """Config 4: 1,048,576 x M = 10 (2.0 GB of coefficients) in one multi-device call."""
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    B, M = B_FULL, 10
    so, W, T = S.uniform_batch(B, M)
    Wf, Tf = W.reshape(-1, 3), T.reshape(-1)
    dso = torch.from_numpy(so).cuda()
    dW, dT = torch.from_numpy(Wf).cuda(), torch.from_numpy(Tf).cuda()
    dC = torch.full((B * M, 3, 8), float("nan"), dtype=torch.float64, device="cuda")
    dS = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    multi.solve_batch_multi_device(so, dso, dW, dT, dC, dS)
    torch.cuda.synchronize()
    assert int((dS != 0).sum()) == 0
    check_spline_properties_torch(so, dW, dT, dC)
    # bit equality with the single-device uniform entry point on the same batch
    ref = torch.empty_like(dC)
    solver.solve_uniform_device(B, M, dW, dT, ref)
    torch.cuda.synchronize()
    assert torch.equal(dC, ref)
    del ref
    for lo, hi in _slices(so):
        so_l = (so[lo:hi + 1] - so[lo]).astype(np.int32)
        R, rst = oracle.solve_batch(so_l, W[lo:hi].reshape(-1, 3), T[lo:hi].reshape(-1), None, oracle.KKT_C4)
        assert (rst == 0).all()
        C = dC[lo * M:hi * M].cpu().numpy()
        assert batch_rel_err(so_l, C, R) <= TOL, (lo, hi)


def test_config5_full_size(solver, oracle, multi):
    """Config 5: 1,048,576 ragged (M ~ U{2..16}), 10 refinement steps + final solve in
    one tgms_refine_loop_multi_device call."""
    import torch
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(B_FULL, 2, 16)
    B, Sg = len(so) - 1, int(so[-1])
    k_T, eta, iters = 1.0, 0.1, 10
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    dso, dW = d(so), d(W)
    outs = []
    for fn in (multi.refine_loop_multi_device, solver.refine_loop_device):
        dT = d(T.copy())
        dC = torch.full((Sg, 3, 8), float("nan"), dtype=torch.float64, device="cuda")
        dcost = torch.full((B,), float("nan"), dtype=torch.float64, device="cuda")
        dst = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        fn(so, dso, dW, dT, k_T, eta, iters, dC, dcost, dst)
        torch.cuda.synchronize()
        outs.append((dT, dC, dcost, dst))
        if len(outs) == 1:
            assert int((dst != 0).sum()) == 0
            assert bool(torch.isfinite(dcost).all()) and bool((dcost > 0).all())
            check_spline_properties_torch(so, dW, dT, dC)
    for a, b in zip(*outs):  # the multi pipeline == the single-device call, bit for bit
        assert torch.equal(a, b)
    dT, dC, dcost, _ = outs[0]
    del outs
    Tg = dT.cpu().numpy()
    assert not np.array_equal(Tg, T)
    cg = dcost.cpu().numpy()
    for lo, hi in _slices(so):
        so_l, W_l, T_l, _ = SH.shard_csr(so, W, T, None, lo, hi)
        To, co, Co, sto = oracle.refine_batch(so_l, W_l, T_l, None, k_T, eta, iters, oracle.REDUCED)
        assert (sto == 0).all()
        s0, s1 = int(so[lo]), int(so[hi])
        assert np.abs(Tg[s0:s1] / To - 1).max() <= REFINE_TOL_MAX, (lo, hi)
        assert np.abs(cg[lo:hi] / co - 1).max() <= REFINE_TOL_MAX, (lo, hi)
        Cg = dC[s0:s1].cpu().numpy()
        R, rst = oracle.solve_batch(so_l, W_l, Tg[s0:s1], None, oracle.REDUCED)
        assert (rst == 0).all()
        assert batch_rel_err(so_l, Cg, R) <= TOL, (lo, hi)
