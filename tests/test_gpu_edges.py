"""GPU edge cases of the solve, for every method: empty and single-trajectory batches,
stationary goals (all waypoints equal), the largest M at swarm scale, and a ragged
batch whose groups include one-trajectory groups.  Tolerance as everywhere: norm-wise
per (trajectory, axis) <= 1e-9 against the oracle."""
import numpy as np
import pytest

from conftest import batch_rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-9


def _methods():
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_DENSE_KKT, METHOD_REDUCED
    return [METHOD_REDUCED, METHOD_DENSE_KKT, METHOD_BAND_KKT]


@pytest.fixture(params=[0, 1, 2], ids=["reduced", "dense", "band"])
def method(request, solver):
    solver.set_method(_methods()[request.param])
    yield request.param
    solver.set_method(_methods()[0])


def test_empty_batch(solver, method):
    import torch
    C, st, worst = solver.solve(np.zeros(1, np.int32), np.zeros((0, 3)), np.zeros(0))
    assert worst == 0 and C.shape == (0, 3, 8) and st.shape == (0,)
    e = torch.empty((0,), dtype=torch.float64, device="cuda")
    solver.solve_uniform_device(0, 3, e, e, e, None)  # no launch, no error


@pytest.mark.parametrize("M", [1, 3, 10])
def test_single_trajectory(solver, oracle, method, M):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(1, M, seed=5000 + M)
    C, st, worst = solver.solve(so, W.reshape(-1, 3), T.reshape(-1))
    assert worst == 0 and st[0] == 0
    R, _ = oracle.solve_batch(so, W.reshape(-1, 3), T.reshape(-1), None, oracle.KKT_C4)
    assert batch_rel_err(so, C, R) <= TOL


def test_stationary_goal(solver, method):
    """All waypoints equal, rest to rest: the optimum is the constant polynomial, so every
    coefficient but c0 is exactly 0 and c0 is the waypoint."""
    B, M = 40, 6
    so = np.arange(B + 1, dtype=np.int32) * M
    W = np.repeat(np.random.default_rng(1).uniform(-5, 5, size=(B, 1, 3)), M + 1, axis=1).reshape(-1, 3)
    T = np.random.default_rng(2).uniform(0.5, 3.0, size=B * M)
    C, st, worst = solver.solve(so, W, T)
    assert worst == 0
    C = C.reshape(B, M, 3, 8)
    assert np.abs(C[..., 1:]).max() <= 1e-9
    w0 = W.reshape(B, M + 1, 3)[:, :1, :]
    assert np.abs(C[..., 0] - w0).max() <= 1e-9 * np.abs(w0).max()


def test_ragged_single_member_groups(solver, oracle, method):
    """Every M group holds one trajectory (one partially filled wavefront per group)."""
    from trajectory_generator_ros2_amd import synthetic as S
    hi = 10 if method == 1 else 16
    Ms = np.arange(1, hi + 1)
    so = np.concatenate([[0], np.cumsum(Ms)]).astype(np.int32)
    rng = np.random.default_rng(6000)
    W = np.concatenate([S.uniform_batch(1, int(m), seed=6000 + int(m))[1].reshape(-1, 3) for m in Ms])
    T = np.concatenate([S.uniform_batch(1, int(m), seed=6000 + int(m))[2].reshape(-1) for m in Ms])
    perm = rng.permutation(len(Ms))  # groups not in M order in the batch
    so_p = np.concatenate([[0], np.cumsum(Ms[perm])]).astype(np.int32)
    W_p = np.concatenate([W[so[b] + b: so[b + 1] + b + 1] for b in perm])
    T_p = np.concatenate([T[so[b]: so[b + 1]] for b in perm])
    C, st, worst = solver.solve(so_p, W_p, T_p)
    assert worst == 0 and (st == 0).all()
    R, _ = oracle.solve_batch(so_p, W_p, T_p, None, oracle.REDUCED)
    assert batch_rel_err(so_p, C, R) <= TOL


def test_largest_m_at_swarm_scale(solver, oracle):
    """M = 16 (the largest supported) for 131,072 trajectories (config-4 shard size, 403 MB
    of coefficients) through the device API, reduced and band methods: the first and last
    256 trajectories against the oracle, every status OK, the two methods agree on all."""
    import torch
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    B, M = 131072, 16
    so, W, T = S.uniform_batch(B, M, seed=7000)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    out = {}
    for meth in (METHOD_REDUCED, METHOD_BAND_KKT):
        solver.set_method(meth)
        dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
        dS = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        solver.solve_uniform_device(B, M, dW, dT, dC, dS)
        torch.cuda.synchronize()
        assert int((dS != 0).sum()) == 0
        out[meth] = dC
    solver.set_method(METHOD_REDUCED)
    err = (out[METHOD_BAND_KKT] - out[METHOD_REDUCED]).abs().amax(dim=(1, 3)) / \
        out[METHOD_REDUCED].abs().amax(dim=(1, 3))
    assert float(err.max()) <= TOL
    for sl in (slice(0, 256), slice(B - 256, B)):
        sub_so = (np.arange(257, dtype=np.int32) * M)
        R, _ = oracle.solve_batch(sub_so, W[sl].reshape(-1, 3), T[sl].reshape(-1), None, oracle.REDUCED)
        C = out[METHOD_BAND_KKT][sl].reshape(-1, 3, 8).cpu().numpy()
        assert batch_rel_err(sub_so, C, R) <= TOL


@pytest.mark.parametrize("t_small", [1e-100, 1e-200])
def test_breakdown_writes_exact_zeros(solver, method, t_small):
    """A segment time so small that its powers underflow makes the KKT numerically
    singular (the oracle's LU reports TGMS_ERR_SINGULAR from 1e-100 on).  Whatever a
    method reports for such a trajectory, a failed one must come out as exact zeros
    (never stale or NaN data from the caller's buffer), and its neighbours must be
    untouched by it."""
    from trajectory_generator_ros2_amd import ERR_NONFINITE, ERR_SINGULAR, OK
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(3, 2, seed=77)
    W, T = W.reshape(-1, 3), T.reshape(-1).copy()
    T[3] = t_small  # trajectory 1, second segment
    C = np.full((6, 3, 8), np.nan)
    st = np.full(3, -1, np.int32)
    _, st, worst = solver.solve(so, W, T, out=(C, st))
    assert st[0] == OK and st[2] == OK
    assert st[1] in (OK, ERR_SINGULAR, ERR_NONFINITE)
    if st[1] in (ERR_SINGULAR, ERR_NONFINITE):  # every failure status: exact zeros
        assert (C[2:4] == 0.0).all(), C[2:4]
    assert np.isfinite(C[[0, 1, 4, 5]]).all()


@pytest.mark.parametrize("M", [2, 3, 10])
def test_overflow_reports_nonfinite_and_writes_zeros(solver, method, M):
    """Finite inputs whose solution overflows (waypoints near DBL_MAX): the trajectory is
    reported TGMS_ERR_NONFINITE and comes out as exact zeros, like every other failure
    (the emit gate used to cover only invalid and singular trajectories); its
    neighbours are unaffected.  Even M goes through the lane kernel (uniform, reduced),
    odd M through the lane-pair kernel, every method through its own kernel; the ragged
    form covers the grouped paths."""
    from trajectory_generator_ros2_amd import ERR_NONFINITE, ERR_SINGULAR, OK
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(5, M, seed=78 + M)
    W, T = W.reshape(-1, 3).copy(), T.reshape(-1).copy()
    # trajectory 2: waypoints near the top of the range and short segments, so the exact
    # solution's higher coefficients (~ dw 35 / T^4) exceed DBL_MAX whatever the method
    W[2 * (M + 1): 3 * (M + 1)] *= 1e306
    T[2 * M: 3 * M] = 0.01
    assert np.isfinite(W).all()
    for ragged in (False, True):
        so_r = so
        W_r, T_r = W, T
        if ragged:  # append a 1-segment trajectory: the batch is no longer uniform
            so_r = np.concatenate([so, [so[-1] + 1]]).astype(np.int32)
            W_r = np.concatenate([W, [[0, 0, 1], [1, 1, 1]]])
            T_r = np.concatenate([T, [1.0]])
        C = np.full((int(so_r[-1]), 3, 8), np.nan)
        st = np.full(len(so_r) - 1, -1, np.int32)
        _, st, _ = solver.solve(so_r, W_r, T_r, out=(C, st))
        assert st[2] in (ERR_NONFINITE, ERR_SINGULAR), (ragged, st)
        assert (C[2 * M: 3 * M] == 0.0).all(), C[2 * M: 3 * M]
        others = [b for b in range(len(so_r) - 1) if b != 2]
        assert (st[others] == OK).all(), st
        for b in others:
            assert np.isfinite(C[so_r[b]: so_r[b + 1]]).all()


def test_ragged_nan_end_derivative_is_invalid(solver, oracle):
    """A non-finite end derivative is a non-finite input (include/tgms.h): on the ragged
    lane-pair paths (every M class) the trajectory is flagged TGMS_ERR_INVALID_ARG and comes
    out as exact zeros, and the refinement loop leaves its times alone; the other
    trajectories are unaffected (bit-equal to the batch with the NaNs replaced)."""
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    solver.set_method(METHOD_REDUCED)
    rng = np.random.default_rng(5150)
    so, W, T = S.ragged_batch(1200, 1, 16, seed=5150)
    B = len(so) - 1
    M = np.diff(so)
    ED = rng.normal(size=(B, 18))
    bad = [int(np.flatnonzero(M == m)[1]) for m in (1, 2, 7, 11, 12, 13, 14, 16)]
    ED_ok = ED.copy()
    for i, b in enumerate(bad):
        ED[b, (5 * i) % 18] = np.nan if i % 2 else np.inf
    C, st, worst = solver.solve(so, W, T, ED)
    assert worst == ERR_INVALID_ARG
    assert all(st[b] == ERR_INVALID_ARG for b in bad)
    good = np.setdiff1d(np.arange(B), bad)
    assert (st[good] == 0).all()
    for b in bad:
        assert (C[so[b]:so[b + 1]] == 0.0).all()
    C2, _, _ = solver.solve(so, W, T, ED_ok)
    for b in good:
        assert np.array_equal(C[so[b]:so[b + 1]], C2[so[b]:so[b + 1]])
    R, _ = oracle.solve_batch(so, W, T, ED_ok, oracle.REDUCED)
    for b in good[:200]:
        sl = slice(so[b], so[b + 1])
        assert batch_rel_err([0, so[b + 1] - so[b]], C[sl], R[sl]) <= TOL
    # the refinement loop: the invalid trajectories keep their times and come out as zeros
    T1, C1, cost1, st1, w1 = solver.refine(so, W, T, ED, iters=10)
    T2, C2, cost2, st2, _ = solver.refine(so, W, T, ED_ok, iters=10)
    assert w1 == ERR_INVALID_ARG
    assert all(st1[b] == ERR_INVALID_ARG for b in bad)
    assert (st1[good] == 0).all()
    for b in bad:
        assert np.array_equal(T1[so[b]:so[b + 1]], np.asarray(T).reshape(-1)[so[b]:so[b + 1]])
        assert (C1[so[b]:so[b + 1]] == 0.0).all()
    for b in good:
        assert np.array_equal(T1[so[b]:so[b + 1]], T2[so[b]:so[b + 1]])
        assert np.array_equal(C1[so[b]:so[b + 1]], C2[so[b]:so[b + 1]])
        assert cost1[b] == cost2[b]
