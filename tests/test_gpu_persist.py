"""The refinement loop's persistent one-wave class (k_refine_loop_dev, round 6).

When a ragged batch has more one-wave tiles (32 trajectories of M above the occupancy
boundary) than the GPU has SIMDs, k_plan_scatter sizes that class as persistent waves that
take tiles from a counter in the device plan.  A tile's arithmetic does not depend on which
wave runs it, so the result must be bit-identical to the same trajectories refined in chunks
small enough for one block per tile -- times, costs, coefficients and statuses -- with and
without end derivatives (whose class boundary is lower: M >= 12)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 16384  # <= ~180 one-wave tiles per chunk: one block per tile


@pytest.mark.parametrize("with_ed", [False, True], ids=["rest", "end_derivs"])
def test_persistent_class_bit_equal_to_chunked_calls(solver, with_ed):
    import torch
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    B = 196608
    so, W, T = S.ragged_batch(B, 2, 16, seed=4242)
    ED = np.random.default_rng(7).normal(0.0, 0.5, size=(B, 18)) if with_ed else None
    boundary = 11 if with_ed else 13  # TGMS_TWO_WAVE_MAX_M(_ED)
    Ms = np.diff(so)
    tiles1 = sum(-(-int((Ms == m).sum()) // 32) for m in range(boundary + 1, 17))
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    assert tiles1 > simds, (tiles1, simds)  # the whole batch takes the persistent path
    k_T, eta, iters = 1.0, 0.1, 10
    d = lambda x: None if x is None else torch.from_numpy(np.ascontiguousarray(x)).cuda()

    def run(so_, W_, T_, ED_):
        Bn, Sn = len(so_) - 1, int(so_[-1])
        dT = d(T_.copy())
        dC = torch.full((Sn, 3, 8), float("nan"), dtype=torch.float64, device="cuda")
        dcost = torch.full((Bn,), float("nan"), dtype=torch.float64, device="cuda")
        dst = torch.full((Bn,), -1, dtype=torch.int32, device="cuda")
        solver.refine_loop_device(so_, d(so_), d(W_), dT, k_T, eta, iters, dC, dcost, dst, d_end_derivs=d(ED_))
        torch.cuda.synchronize()
        return dT, dC, dcost, dst

    whole = run(so, W, T, ED)
    assert int((whole[3] != 0).sum()) == 0
    assert bool(torch.isfinite(whole[1]).all())
    for lo in range(0, B, CHUNK):
        hi = min(B, lo + CHUNK)
        so_l, W_l, T_l, ED_l = SH.shard_csr(so, W, T, ED, lo, hi)
        part = run(so_l, W_l, T_l, ED_l)
        s0, s1 = int(so[lo]), int(so[hi])
        assert torch.equal(part[0], whole[0][s0:s1]), lo
        assert torch.equal(part[1], whole[1][s0:s1]), lo
        assert torch.equal(part[2], whole[2][lo:hi]), lo
        assert torch.equal(part[3], whole[3][lo:hi]), lo
