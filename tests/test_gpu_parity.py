"""GPU parity: libtgms (HIP, gfx950) through its C ABI vs the oracle and the exact goldens.

Tolerance (BASELINE.json north_star): per (trajectory, axis),
norm-wise  ||c_gpu - c_ref||_inf / ||c_ref||_inf <= 1e-9.  Element-wise relative
error is not used: rest-to-rest segments have exact zero coefficients.
"""
import os

import numpy as np
import pytest

from conftest import (batch_rel_err, check_spline_properties, gradient_rel_err, load_refine_golden,
                      recovered_gradient, solve_goldens)

pytestmark = pytest.mark.gpu

TOL = 1e-9
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _uniform(B, M, seed):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(B, M, seed=seed)
    return so, W.reshape(-1, 3), T.reshape(-1)


def _methods():
    from trajectory_generator_ros2_amd import METHOD_DENSE_KKT, METHOD_REDUCED
    return [METHOD_REDUCED, METHOD_DENSE_KKT]


@pytest.mark.parametrize("M", list(range(1, 17)))
def test_reduced_uniform_vs_oracle(solver, oracle, M):
    so, W, T = _uniform(257, M, seed=100 + M)  # 257: last wavefront partially filled
    C, st, worst = solver.solve(so, W, T)
    assert worst == 0 and (st == 0).all()
    R, rst = oracle.solve_batch(so, W, T, None, oracle.KKT_C4 if M <= 10 else oracle.REDUCED)
    assert (rst == 0).all()
    assert batch_rel_err(so, C, R) <= TOL


@pytest.mark.parametrize("M", [1, 2, 3, 5, 10])
def test_dense_kkt_uniform_vs_oracle(solver, oracle, M):
    from trajectory_generator_ros2_amd import METHOD_DENSE_KKT, METHOD_REDUCED
    so, W, T = _uniform(130, M, seed=200 + M)
    solver.set_method(METHOD_DENSE_KKT)
    try:
        C, st, worst = solver.solve(so, W, T)
    finally:
        solver.set_method(METHOD_REDUCED)
    assert worst == 0 and (st == 0).all()
    R, _ = oracle.solve_batch(so, W, T, None, oracle.KKT_C4)
    assert batch_rel_err(so, C, R) <= TOL


@pytest.mark.parametrize("method", [0, 1])
def test_end_derivs_vs_oracle(solver, oracle, method):
    rng = np.random.default_rng(5)
    M = 6 if method == 1 else 9
    so, W, T = _uniform(200, M, seed=300)
    ED = rng.normal(size=(200, 18))
    solver.set_method(method)
    try:
        C, st, worst = solver.solve(so, W, T, ED)
    finally:
        solver.set_method(0)
    assert worst == 0
    R, _ = oracle.solve_batch(so, W, T, ED, oracle.KKT_C4)
    assert batch_rel_err(so, C, R) <= TOL


@pytest.mark.parametrize("method", [0, 1])
def test_ragged_vs_oracle(solver, oracle, method):
    from trajectory_generator_ros2_amd import synthetic as S
    hi = 16 if method == 0 else 10
    so, W, T = S.ragged_batch(1000, 1, hi, seed=400 + method)
    solver.set_method(method)
    try:
        C, st, worst = solver.solve(so, W, T)
    finally:
        solver.set_method(0)
    assert worst == 0 and (st == 0).all()
    R, _ = oracle.solve_batch(so, W, T, None, oracle.REDUCED)
    assert batch_rel_err(so, C, R) <= TOL


def test_ragged_mixed_classes_end_derivs_and_invalid(solver, oracle):
    """One ragged batch spanning both launch classes of the fused ragged kernels
    (M <= 11 and M >= 12, every M in 1..16), with end derivatives and a few invalid
    trajectories in different groups: valid ones match the oracle, invalid ones are
    flagged, nothing leaks across groups."""
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG
    from trajectory_generator_ros2_amd import synthetic as S
    rng = np.random.default_rng(77)
    so, W, T = S.ragged_batch(700, 1, 16, seed=77)
    B = len(so) - 1
    ED = rng.normal(size=(B, 18))
    T = T.copy()
    M = np.diff(so)
    bad = [int(np.flatnonzero(M == m)[0]) for m in (1, 7, 11, 12, 16)]
    for b in bad:
        T[so[b] + M[b] - 1] = -0.5
    C, st, worst = solver.solve(so, W, T, ED)
    assert worst == ERR_INVALID_ARG
    assert all(st[b] == ERR_INVALID_ARG for b in bad)
    good = np.setdiff1d(np.arange(B), bad)
    assert (st[good] == 0).all()
    T2 = T.copy()
    for b in bad:
        T2[so[b] + M[b] - 1] = 1.0
    R, _ = oracle.solve_batch(so, W, T2, ED, oracle.REDUCED)
    for b in good:
        c, r = C[so[b]:so[b + 1]], R[so[b]:so[b + 1]]
        for a in range(3):
            assert np.abs(c[:, a] - r[:, a]).max() <= TOL * max(np.abs(r[:, a]).max(), 1e-300)
    assert np.isfinite(C).all()


@pytest.mark.parametrize("path", solve_goldens())
@pytest.mark.parametrize("method", [0, 1])
def test_goldens_exact(solver, path, method):
    g = np.load(path)
    so = g["seg_offsets"]
    if method == 1 and int(np.diff(so).max()) > 10:
        pytest.skip("dense KKT supports M <= 10")
    ED = g["end_derivs"] if "end_derivs" in g.files else None
    solver.set_method(method)
    try:
        C, st, worst = solver.solve(so, g["waypoints"], g["seg_times"], ED)
    finally:
        solver.set_method(0)
    assert worst == 0
    assert batch_rel_err(so, C, g["coeffs"]) <= TOL


def test_invalid_inputs(solver):
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, ERR_UNSUPPORTED
    so, W, T = _uniform(70, 4, seed=7)
    T = T.copy(); W = W.copy()
    T[4 * 3 + 1] = 0.0        # trajectory 3: T <= 0
    T[4 * 5] = -1.0           # trajectory 5
    W[(4 + 1) * 9 + 2, 1] = np.nan  # trajectory 9: NaN waypoint
    T[4 * 66 + 3] = np.inf    # trajectory 66 (second wavefront)
    for method in (0, 1):
        solver.set_method(method)
        C, st, worst = solver.solve(so, W, T)
        bad = {3, 5, 9, 66}
        assert worst == ERR_INVALID_ARG
        assert all(st[b] == ERR_INVALID_ARG for b in bad)
        assert all(st[b] == 0 for b in range(70) if b not in bad)
        assert np.isfinite(C).all()
    solver.set_method(0)
    # structural errors are reported by the host before any launch
    _, _, w = solver.solve(np.array([0, 0], np.int32), np.zeros((1, 3)), np.zeros(0))
    assert w == ERR_INVALID_ARG
    so17, W17, T17 = _uniform(2, 17, seed=1)
    assert solver.solve(so17, W17, T17)[2] == ERR_INVALID_ARG
    so11, W11, T11 = _uniform(2, 11, seed=1)
    solver.set_method(1)
    assert solver.solve(so11, W11, T11)[2] == ERR_UNSUPPORTED
    solver.set_method(0)


def test_ragged_structural_errors_name_the_first_trajectory(solver):
    """Ragged offsets are validated on the host in chunks (csrc/tgms_capi.hip check_offsets);
    an error must still name the FIRST offending trajectory, with the status a sequential
    scan gives: M outside 1..16 -> TGMS_ERR_INVALID_ARG, M above the method's limit ->
    TGMS_ERR_UNSUPPORTED, whichever comes first."""
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, ERR_UNSUPPORTED, METHOD_DENSE_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(4001, 2, 9, seed=31)
    M = np.diff(so).astype(np.int64)
    for bad_b, bad_m, status in ((2999, 0, ERR_INVALID_ARG), (1500, 17, ERR_INVALID_ARG), (7, -3, ERR_INVALID_ARG)):
        M2 = M.copy()
        M2[bad_b] = bad_m
        M2[3500] = 0  # a later offender: not the one reported
        so2 = np.concatenate([[0], np.cumsum(M2)]).astype(np.int32)
        _, _, w = solver.solve(so2, np.zeros((int(so2[-1]) + len(M2), 3)), np.ones(max(int(so2[-1]), 1)))
        assert w == status
        assert f"trajectory {bad_b} has {bad_m} segments" in solver.last_error(), solver.last_error()
    # the dense KKT stops at M = 10: the first trajectory above it is named
    M2 = M.copy()
    M2[1234] = 12
    M2[2345] = 17  # invalid, but after the unsupported one
    so2 = np.concatenate([[0], np.cumsum(M2)]).astype(np.int32)
    solver.set_method(METHOD_DENSE_KKT)
    try:
        _, _, w = solver.solve(so2, np.zeros((int(so2[-1]) + len(M2), 3)), np.ones(int(so2[-1])))
    finally:
        solver.set_method(METHOD_REDUCED)
    assert w == ERR_UNSUPPORTED
    assert "trajectory 1234 has 12 segments" in solver.last_error(), solver.last_error()
    # and a valid ragged batch of the same size still solves (the chunked grouping is exact)
    C, st, w = solver.solve(so, W, T)
    assert w == 0 and (st == 0).all()


def test_config3_full_size_properties(solver, oracle):
    """BASELINE config 3 at full size (B = 65,536, M = 10) through the device API:
    parity with the oracle on every trajectory + size-independent properties."""
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    B, M = 65536, 10
    so, W, T = S.uniform_batch(B, M)
    dW = torch.from_numpy(W).cuda()
    dT = torch.from_numpy(T).cuda()
    dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
    dS = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    C = dC.cpu().numpy().reshape(-1, 3, 8)
    assert (dS.cpu().numpy() == 0).all()
    R, _ = oracle.solve_batch(so, W.reshape(-1, 3), T.reshape(-1), None, oracle.REDUCED)
    assert batch_rel_err(so, C, R) <= TOL
    # interpolation and C6 continuity at every interior knot, rest at both ends
    check_spline_properties(so, W.reshape(-1, 3), T.reshape(-1), C)


@pytest.mark.parametrize("M", [12, 13, 14, 16])
def test_uniform_large_m_full_size_every_trajectory(solver, oracle, M):
    """Round 5: the whole-line lane-pair kernel (even M >= 12) and the axis-sequential one
    (odd M) at the bench's size, 65,536 trajectories, every trajectory against the oracle at
    1e-9, over three back-to-back launches into the same buffer with different inputs (a
    stale store offset would leave another launch's or another trajectory's values behind;
    the band kernel's store-offset failure)."""
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    B = 65536
    dC = torch.full((B, M, 3, 8), float("nan"), dtype=torch.float64, device="cuda")
    dS = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    for rep in range(3):
        so, W, T = S.uniform_batch(B, M, seed=900 + 10 * M + rep)
        dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
        solver.solve_uniform_device(B, M, dW, dT, dC, dS)
        torch.cuda.synchronize()
        assert (dS.cpu().numpy() == 0).all()
        R, rst = oracle.solve_batch(so, W.reshape(-1, 3), T.reshape(-1), None, oracle.REDUCED)
        assert (rst == 0).all()
        assert batch_rel_err(so, dC.cpu().numpy().reshape(-1, 3, 8), R) <= TOL, rep


def test_device_ragged_matches_host(solver):
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(5000, 2, 16, seed=9)
    C_host, st, worst = solver.solve(so, W, T)
    assert worst == 0
    dso = torch.from_numpy(so).cuda()
    dC = torch.zeros((int(so[-1]), 3, 8), dtype=torch.float64, device="cuda")
    solver.solve_batch_device(so, dso, torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda(), dC,
                              stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(dC.cpu().numpy(), C_host)


def test_sampler_vs_oracle(solver, oracle):
    from trajectory_generator_ros2_amd import YAW_VELOCITY
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(40, 1, 16, seed=12)
    C, _, worst = solver.solve(so, W, T)
    assert worst == 0
    for yaw_mode in (0, YAW_VELOCITY):
        offs, out = solver.sample(so, W, T, None, C, 0.01, yaw_mode, 0.3)
        for b in range(40):
            s0, s1 = so[b], so[b + 1]
            ref = oracle.sample(C[s0:s1], T[s0:s1], W[s0 + b:s1 + b + 1], None, 0.01, yaw_mode, 0.3)
            got = out[offs[b]:offs[b + 1]]
            assert got.shape == ref.shape
            for f0, f1 in ((0, 3), (3, 6), (6, 9), (9, 12)):
                scale = max(np.abs(ref[:, f0:f1]).max(), 1e-300)
                assert np.abs(got[:, f0:f1] - ref[:, f0:f1]).max() <= TOL * scale
            assert np.array_equal(got[-1, :12], ref[-1, :12])  # pinned final sample
            sp = np.hypot(ref[:, 3], ref[:, 4])
            m = (sp > 2e-3)
            dpsi = np.angle(np.exp(1j * (got[m, 12] - ref[m, 12])))
            assert np.abs(dpsi).max() <= 1e-9
            m0 = (sp < 5e-4)
            assert np.array_equal(got[m0, 12], ref[m0, 12])


@pytest.mark.parametrize("name", ["c1", "c3_sampled", "end_derivs"])
def test_sampler_vs_exact_golden(solver, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    so = g["seg_offsets"]
    ED = g["end_derivs"] if "end_derivs" in g.files else None
    C, _, worst = solver.solve(so, g["waypoints"], g["seg_times"], ED)
    assert worst == 0
    offs, out = solver.sample(so, g["waypoints"], g["seg_times"], ED, C, float(g["dt"]))
    assert np.array_equal(offs, g["sample_offsets"])
    ref = g["samples"]
    for f0, f1 in ((0, 3), (3, 6), (6, 9), (9, 12)):
        scale = np.abs(ref[:, f0:f1]).max()
        assert np.abs(out[:, f0:f1] - ref[:, f0:f1]).max() <= TOL * scale


def test_sharded_solve_matches_unsharded(solver):
    """§8(e): per-rank shards of a ragged batch solved on the GPU concatenate to the
    unsharded GPU result bit-for-bit (trajectories are independent)."""
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(3001, 1, 16, seed=11)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    C_all, st_all, worst = solver.solve(so, W, T)
    assert worst == 0
    parts, sts = [], []
    for r in range(4):
        sb = SH.ShardedBatch(so, W, T, None, rank=r, world=4)
        C, st = sb.solve(lambda a, b, c, d: solver.solve(a, b, c, d)[:2])
        parts.append(C)
        sts.append(st[: sb.hi - sb.lo])
    np.testing.assert_array_equal(np.concatenate(parts), C_all)
    np.testing.assert_array_equal(np.concatenate(sts), st_all[:3001])


@pytest.mark.parametrize("ragged", [False, True])
def test_refine_matches_oracle(solver, oracle, ragged):
    """Config-5 time refinement (10 steps + final solve) on the GPU vs the oracle's
    restatement of the same step, at north_star's 1e-9 (round 6: measured <= 2.9e-11 with
    the displacement-form oracle; round 5's oracle gradient was ~1e-8 off exact and this
    bound stood at 1e-8)."""
    from trajectory_generator_ros2_amd import synthetic as S
    if ragged:
        so, W, T = S.ragged_batch(257, 1, 16, seed=21)
    else:
        so, W, T = S.uniform_batch(257, 10, seed=21)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    Tg, Cg, cg, stg, worst = solver.refine(so, W, T, None, 1.0, 0.1, 10)
    To, co, Co, sto = oracle.refine_batch(so, W, T, None, 1.0, 0.1, 10, oracle.REDUCED)
    assert worst == 0 and (sto == 0).all()
    assert np.abs(Tg / To - 1).max() <= TOL
    assert np.abs(cg / co - 1).max() <= TOL
    assert batch_rel_err(so, Cg, Co) <= TOL
    assert not np.array_equal(Tg, T)


def _step_gradient_from_coeffs(C, W, T, ED, kT):
    """The refinement step's gradient formula (csrc/tgms_reduced.hip seg_cost_p: the snap
    cost's T-derivative from the scaled monomial data P4..P7, r = 1/T) evaluated in numpy on
    a solve's own knot data: segment i's start (v, a, j) from its coefficients, its end data
    from the next segment's start (the shared knot) or the final end derivatives."""
    M = T.shape[0]
    out = np.zeros(M)
    for i in range(M):
        r = 1.0 / T[i]
        r2, r3 = r * r, r * r * r
        for a in range(3):
            c = C[i, a]
            v0, a0, j0 = c[1], 2.0 * c[2], 6.0 * c[3]
            if i + 1 < M:
                cn = C[i + 1, a]
                v1, a1 = cn[1], 2.0 * cn[2]
            else:
                v1, a1 = (ED[9 + a], ED[12 + a]) if ED is not None else (0.0, 0.0)
            D = (W[i + 1, a] - W[i, a]) * r3
            V0, A0, V1, A1 = v0 * r2, a0 * r, v1 * r2, a1 * r
            P = [c[4] / r, c[5] / r2, c[6] / r3, c[7] / (r2 * r2)]
            Qv = [105.0 * D - 40.0 * V0 - 5.0 * A0 - 30.0 * V1 + 2.5 * A1,
                  -252.0 * D + 90.0 * V0 + 10.0 * A0 + 78.0 * V1 - 7.0 * A1,
                  210.0 * D - 72.0 * V0 - 7.5 * A0 - 68.0 * V1 + 6.5 * A1,
                  -60.0 * D + 20.0 * V0 + 2.0 * A0 + 20.0 * V1 - 2.0 * A1]
            Hm = np.array([[576.0, 1440.0, 2880.0, 5040.0], [1440.0, 4800.0, 10800.0, 20160.0],
                           [2880.0, 10800.0, 25920.0, 50400.0], [5040.0, 20160.0, 50400.0, 100800.0]])
            HP = Hm @ np.array(P)
            Q = float(np.dot(P, HP))
            G = float(np.dot(Qv, HP))
            out[i] += r2 * -(Q + 2.0 * G)
    return out


@pytest.mark.parametrize("ragged", [False, True])
@pytest.mark.parametrize("with_ed", [False, True])
def test_refine_one_step_at_north_star_tolerance(solver, oracle, ragged, with_ed):
    """ONE refinement step (iters = 1) on 257 trajectories against the oracle at north_star's
    1e-9 with no iteration to amplify rounding: the new times T_1, the cost at the input
    times (iters = 0) and at T_1, the coefficients at T_1, each norm-wise per trajectory.
    The per-segment gradient dJ_i/dT_i the step applied, recovered from
    T_1 = T_0 exp(-eta T_0 (dJ + k_T) / F) (unclamped segments), is held at 1e-9
      - to the step's formula evaluated in numpy on the GPU's own solve at T_0: the step is
        exactly its formula on its solve;
      - to the EXACT gradient of these same inputs (tests/golden/refine_grad.npz groups u257,
        u257e, r257, r257e: rational solve and rational dJ_i/dT_i, oracle/exact.py).
    The fp64 oracle's own gradient is not the reference here: on r257e it is itself up to
    8.2e-10 off exact (its dense Cholesky's knot data, ~2e-11, amplified ~30x by the
    gradient; tests/test_refine_oracle.py holds it to the same fixture at 1e-9), so GPU vs
    oracle would charge the oracle's error to the GPU (round 5 stood at 1e-6 for that reason).
    Uniform batches run the step kernels, ragged ones the fused loop."""
    from trajectory_generator_ros2_amd import synthetic as S
    if ragged:
        so, W, T = S.ragged_batch(257, 1, 16, seed=61)
    else:
        so, W, T = S.uniform_batch(257, 10, seed=62)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    B = len(so) - 1
    ED = np.random.default_rng(63).normal(scale=0.3, size=(B, 18)) if with_ed else None
    k_T, eta, groups = load_refine_golden()
    fx = groups[("r257" if ragged else "u257") + ("e" if with_ed else "")]
    assert np.array_equal(fx["seg_times"], T) and np.array_equal(fx["waypoints"], W)
    assert (k_T, eta) == (1.0, 0.02)
    _, C0, F0, st0, w0 = solver.refine(so, W, T, ED, k_T, eta, 0)
    T1, C1, F1, st1, w1 = solver.refine(so, W, T, ED, k_T, eta, 1)
    assert w0 == 0 and w1 == 0 and (st0 == 0).all() and (st1 == 0).all()
    To, Fo, Co, sto = oracle.refine_batch(so, W, T, ED, k_T, eta, 1, oracle.REDUCED)
    assert (sto == 0).all()
    assert np.abs(T1 / To - 1).max() <= TOL
    assert np.abs(F1 / Fo - 1).max() <= TOL
    assert batch_rel_err(so, C1, Co) <= TOL
    assert np.abs(F0 / fx["F"] - 1).max() <= 1e-11
    assert np.abs(T1 / fx["T1"] - 1).max() <= 1e-11
    g, free = recovered_gradient(T, T1, np.repeat(F0, np.diff(so)), k_T, eta)
    assert free.mean() >= 0.9
    mine = np.concatenate([_step_gradient_from_coeffs(C0[so[b]:so[b + 1]], W[so[b] + b:so[b + 1] + b + 1],
                                                      T[so[b]:so[b + 1]], None if ED is None else ED[b], k_T)
                           for b in range(B)])
    assert gradient_rel_err(so, g, mine, free) <= TOL
    assert gradient_rel_err(so, g, fx["dJ"], free) <= TOL


@pytest.mark.parametrize("group", ["u10", "u10e", "u7e", "u16", "r", "re", "u257", "u257e", "r257", "r257e"])
def test_refine_step_matches_exact_fixture(solver, group):
    """The config-5 step against EXACT arithmetic (tests/golden/refine_grad.npz, made by
    oracle/exact.py: rational solve, rational J_i and dJ_i/dT_i, mpmath exp): the GPU's
    F(T_0) and T_1 within 1e-11, and the gradient it applied (recovered from T_1, a recovery
    the CPU test test_gradient_recovery_is_exact_enough holds to 1e-11) within 1e-9 of the
    exact dJ_i/dT_i, norm-wise per trajectory.  Groups: uniform M = 10 / 7 / 16 (step
    kernels) and ragged M = 1..16 (the fused loop), with and without end derivatives."""
    k_T, eta, groups = load_refine_golden()
    d = groups[group]
    so, W, T, ED = d["seg_offsets"], d["waypoints"], d["seg_times"], d["end_derivs"]
    _, _, F0, st0, w0 = solver.refine(so, W, T, ED, k_T, eta, 0, coeffs=False)
    T1, _, _, st1, w1 = solver.refine(so, W, T, ED, k_T, eta, 1, coeffs=False)
    assert w0 == 0 and w1 == 0 and (st0 == 0).all() and (st1 == 0).all()
    assert np.abs(F0 / d["F"] - 1).max() <= 1e-11
    assert np.abs(T1 / d["T1"] - 1).max() <= 1e-11
    g, free = recovered_gradient(T, T1, np.repeat(F0, np.diff(so)), k_T, eta)
    assert free.mean() > 0.9
    assert gradient_rel_err(so, g, d["dJ"], free) <= TOL


def test_refine_device_step_and_errors(solver):
    import torch
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, ERR_UNSUPPORTED, METHOD_DENSE_KKT, TgmsError
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(100, 7, seed=4)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    dT2 = torch.empty_like(dT)
    dcost = torch.empty(100, dtype=torch.float64, device="cuda")
    solver.refine_uniform_device(100, 7, dW, dT, dT2, 1.0, 0.0, dcost)   # eta = 0: same times
    torch.cuda.synchronize()
    assert torch.equal(dT2, dT) and bool((dcost > 0).all())
    with pytest.raises(TgmsError) as e:
        solver.refine_uniform_device(100, 7, dW, dT, dT, 1.0, 0.1)       # aliasing in/out
    assert e.value.status == ERR_INVALID_ARG
    with pytest.raises(TgmsError) as e:
        solver.refine_uniform_device(100, 7, dW, dT, dT2, -1.0, 0.1)     # k_T < 0
    assert e.value.status == ERR_INVALID_ARG
    solver.set_method(METHOD_DENSE_KKT)
    try:
        with pytest.raises(TgmsError) as e:
            solver.refine_uniform_device(100, 7, dW, dT, dT2, 1.0, 0.1)
        assert e.value.status == ERR_UNSUPPORTED
    finally:
        from trajectory_generator_ros2_amd import METHOD_REDUCED
        solver.set_method(METHOD_REDUCED)


def test_refine_loop_device_matches_host(solver):
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(300, 2, 16, seed=8)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    Th, Ch, ch, _, worst = solver.refine(so, W, T, None, 0.5, 0.2, 7)
    assert worst == 0
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    dso, dW, dT = d(so.astype(np.int32)), d(W), d(T.copy())
    dC = torch.empty((int(so[-1]), 3, 8), dtype=torch.float64, device="cuda")
    dcost = torch.empty(300, dtype=torch.float64, device="cuda")
    dst = torch.empty(300, dtype=torch.int32, device="cuda")
    solver.refine_loop_device(so, dso, dW, dT, 0.5, 0.2, 7, dC, dcost, dst)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dT.cpu().numpy(), Th)
    np.testing.assert_array_equal(dC.cpu().numpy(), Ch)
    np.testing.assert_array_equal(dcost.cpu().numpy(), ch)
    assert int(dst.abs().sum()) == 0


@pytest.mark.gpu
def test_device_slices_and_alignment(solver):
    """bench.py's config-4 line solves a batch piece by piece through slices of the
    device arrays: aligned slices give the unsliced result bit for bit; a slice at an
    odd element offset (8-B aligned only) is refused before any launch."""
    import torch
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, TgmsError
    from trajectory_generator_ros2_amd import synthetic as S
    B, M = 4096, 10
    _, W, T = S.uniform_batch(B, M, seed=11)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    full = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
    solver.solve_uniform_device(B, M, dW, dT, full)
    pieces = torch.full_like(full, float("nan"))
    bounds = [0, 64, 1026, 2050, 4096]  # even trajectory offsets: every slice 16-B aligned
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        solver.solve_uniform_device(hi - lo, M, dW[lo:hi], dT[lo:hi], pieces[lo:hi])
    torch.cuda.synchronize()
    assert torch.equal(full, pieces)
    odd = dW.reshape(-1)[1:1 + 100 * (M + 1) * 3]  # 8 bytes past a 16-B boundary
    with pytest.raises(TgmsError) as e:
        solver.solve_uniform_device(100, M, odd, dT[:100], full[:100])
    assert e.value.status == ERR_INVALID_ARG and "aligned" in solver.last_error()


@pytest.mark.parametrize("M", [2, 4, 10, 12, 14, 16, 5, 13])
def test_lane_kernel_end_derivs_invalid_and_tail(solver, oracle, M):
    """Uniform batches with end derivatives on the lane-per-trajectory kernel (even M <= 12)
    and the lane-pair kernel (odd M, M >= 14): a partial last wavefront (B = 3 x 64 + 5;
    for even M the waypoint array has an odd number of doubles, the last one outside
    every 16-B LDS-DMA piece), and invalid trajectories in several wavefronts — T <= 0,
    non-finite T, a NaN waypoint, a NaN end derivative.  Valid trajectories match the
    oracle; invalid ones are flagged TGMS_ERR_INVALID_ARG (a NaN end derivative is a
    non-finite input, include/tgms.h) and come out as exact zeros."""
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG
    B = 3 * 64 + 5
    so, W, T = _uniform(B, M, seed=900 + M)
    assert (W.size % 2) == (M + 1) % 2
    rng = np.random.default_rng(900 + M)
    ED = rng.normal(size=(B, 18))
    T = T.copy(); W = W.copy()
    T[3 * M + M - 1] = 0.0            # trajectory 3: T <= 0 (its last segment)
    T[70 * M] = np.inf                # trajectory 70
    W[130 * (M + 1) + M, 2] = np.nan  # trajectory 130: NaN at its last knot
    ED[B - 1, 17] = np.nan            # last trajectory (tail wavefront): NaN end derivative
    bad = [3, 70, 130, B - 1]
    C, st, worst = solver.solve(so, W, T, ED)
    assert worst == ERR_INVALID_ARG
    assert all(st[b] == ERR_INVALID_ARG for b in bad)
    good = np.setdiff1d(np.arange(B), bad)
    assert (st[good] == 0).all()
    Cb = C.reshape(B, M, 3, 8)
    assert all((Cb[b] == 0.0).all() for b in bad)
    R, rst = oracle.solve_batch(so, W, np.where(np.isfinite(T) & (T > 0), T, 1.0),
                                np.nan_to_num(ED), oracle.REDUCED)
    Rb = R.reshape(B, M, 3, 8)
    for b in good:
        for a in range(3):
            ref = Rb[b, :, a]
            assert np.abs(Cb[b, :, a] - ref).max() <= TOL * max(np.abs(ref).max(), 1e-300)


@pytest.mark.parametrize("method", [0, 2])
def test_two_streams_share_handle_scratch(solver, method):
    """Two ragged solves of one handle issued back to back on two different streams
    (the second call re-uploads the handle's trajectory permutation and, for
    the band method, reuses its U slabs while the first call's kernels may still run).
    The handle orders them on the GPU; both must equal their one-stream host solves."""
    import torch
    from trajectory_generator_ros2_amd import METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    so1, W1, T1 = S.ragged_batch(6000, 2, 16, seed=21)
    so2, W2, T2 = S.ragged_batch(3001, 2, 16, seed=22)  # different B and grouping
    solver.set_method(method)
    try:
        R1, _, w1 = solver.solve(so1, W1, T1)
        R2, _, w2 = solver.solve(so2, W2, T2)
        assert w1 == 0 and w2 == 0
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        dev = [(torch.from_numpy(so).cuda(), torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda(),
                torch.zeros((int(so[-1]), 3, 8), dtype=torch.float64, device="cuda"))
               for so, W, T in ((so1, W1, T1), (so2, W2, T2))]
        torch.cuda.synchronize()
        solver.solve_batch_device(so1, *dev[0], stream=s1.cuda_stream)
        solver.solve_batch_device(so2, *dev[1], stream=s2.cuda_stream)
        torch.cuda.synchronize()
    finally:
        solver.set_method(METHOD_REDUCED)
    assert np.array_equal(dev[0][3].cpu().numpy(), R1)
    assert np.array_equal(dev[1][3].cpu().numpy(), R2)
