"""CPU: the time-allocation refinement math in the oracle.

There is no reference counterpart (the reference has no solver), so the step is
pinned by its own definition:
  - dJ_i/dT_i from the segment's end data (envelope theorem) equals a central
    finite difference of the re-solved optimal cost J(T);
  - the per-segment cost formula equals sum_axes c^T Q c with the survey's a1
    Hessian Q_jk = j!/(j-4)! k!/(k-4)! T^(j+k-7)/(j+k-7);
  - eta = 0 leaves T unchanged; steps lower F on the config-3 data."""
import math

import numpy as np
import pytest

from trajectory_generator_ros2_amd import synthetic as S


def _cost(O, W, T, kT=0.0):
    _, F, C, st = O.refine_times(W, T, None, kT, 0.0, 0, O.KKT_C4)
    assert st == 0
    return F, C


def _q_cost(C, T):
    """survey a1: sum over segments/axes of c^T Q(T) c."""
    J = 0.0
    for i, Ti in enumerate(T):
        for a in range(3):
            c = C[i, a]
            for j in range(4, 8):
                for k in range(4, 8):
                    f = math.factorial(j) / math.factorial(j - 4) * math.factorial(k) / math.factorial(k - 4)
                    J += c[j] * c[k] * f * Ti ** (j + k - 7) / (j + k - 7)
    return J


def test_cost_matches_survey_hessian(oracle):
    _, W, T = S.uniform_batch(4, 5, seed=3)
    for b in range(4):
        F, C = _cost(oracle, W[b], T[b])
        assert abs(F - _q_cost(C, T[b])) <= 1e-10 * F


@pytest.mark.parametrize("M", [1, 2, 3, 6])
def test_gradient_matches_finite_difference(oracle, M):
    """One step with a tiny eta exposes g_i through T_new = T exp(-eta T g / F)."""
    _, W, T = S.uniform_batch(3, M, seed=5)
    kT = 0.7
    for b in range(3):
        F, _ = _cost(oracle, W[b], T[b], kT)
        eta = 1e-9
        Tn, _, _, st = oracle.refine_times(W[b], T[b], None, kT, eta, 1, oracle.KKT_C4)
        assert st == 0
        g = -np.log(Tn / T[b]) * F / (eta * T[b])  # analytic dF/dT_i recovered from the step
        for i in range(M):
            h = 1e-6 * T[b][i]
            Tp, Tm = T[b].copy(), T[b].copy()
            Tp[i] += h
            Tm[i] -= h
            fd = (_cost(oracle, W[b], Tp, kT)[0] - _cost(oracle, W[b], Tm, kT)[0]) / (2 * h)
            assert abs(g[i] - fd) <= 1e-4 * (abs(fd) + kT), (i, g[i], fd)


def test_eta_zero_keeps_times(oracle):
    so, W, T = S.ragged_batch(20, 1, 8, seed=9)
    Tn, cost, _, st = oracle.refine_batch(so, W, T, None, 1.0, 0.0, 5, oracle.REDUCED)
    assert (st == 0).all()
    np.testing.assert_array_equal(Tn, T.reshape(-1))


def test_refinement_lowers_cost(oracle):
    so, W, T = S.uniform_batch(64, 10, seed=2)
    _, c0, _, _ = oracle.refine_batch(so, W, T, None, 1.0, 0.1, 0, oracle.REDUCED)
    Tn, c10, _, st = oracle.refine_batch(so, W, T, None, 1.0, 0.1, 10, oracle.REDUCED)
    assert (st == 0).all()
    assert (c10 <= c0 * (1 + 1e-12)).mean() > 0.95
    assert np.median(c10 / c0) < 0.95
    assert (Tn > 0).all()


@pytest.mark.parametrize("M", [1, 3, 7, 12])
def test_refine_grad_is_the_step_gradient(oracle, M):
    """oracle.refine_grad (the per-segment dJ_i/dT_i and F at fixed times, used to pin one
    GPU step at 1e-9) equals the gradient oracle_refine_times applies, and central finite
    differences of the re-solved cost."""
    rng = np.random.default_rng(40 + M)
    _, W, T = S.uniform_batch(3, M, seed=41 + M)
    kT = 0.3
    for b in range(3):
        ED = rng.normal(size=18) if b == 2 else None
        dJ, F, st = oracle.refine_grad(W[b], T[b], ED, kT, oracle.REDUCED)
        assert st == 0
        eta = 1e-9
        Tn, F0, _, st = oracle.refine_times(W[b], T[b], ED, kT, eta, 1, oracle.REDUCED)
        assert st == 0
        _, Fr, _, _ = oracle.refine_times(W[b], T[b], ED, kT, 0.0, 0, oracle.REDUCED)
        assert F == Fr
        g = -np.log(Tn / T[b]) * F / (eta * T[b]) - kT
        assert np.abs(g - dJ).max() <= 1e-5 * np.abs(dJ).max()
        i = M // 2
        h = 1e-6 * T[b][i]
        Tp, Tm = T[b].copy(), T[b].copy()
        Tp[i] += h
        Tm[i] -= h
        fp = oracle.refine_times(W[b], Tp, ED, kT, 0.0, 0, oracle.REDUCED)[1]
        fm = oracle.refine_times(W[b], Tm, ED, kT, 0.0, 0, oracle.REDUCED)[1]
        assert abs((fp - fm) / (2 * h) - (dJ[i] + kT)) <= 1e-4 * (abs(dJ[i]) + kT)


# ---------------------------------------------------------------- exact pins (round 6)

from fractions import Fraction  # noqa: E402

from conftest import gradient_rel_err, load_refine_golden, recovered_gradient  # noqa: E402


@pytest.mark.parametrize("M", [1, 2, 3])
def test_exact_gradient_is_the_derivative_of_the_exact_cost(M):
    """oracle/exact.py's dJ_i/dT_i (knot data held at the optimum) equals an EXACT central
    difference of the exact optimal cost J*(T) (h = 1e-25 T_i in rationals: the O(h^2)
    truncation is ~1e-50 relative), with and without end derivatives — the envelope theorem
    the refinement step relies on, checked with no rounding anywhere."""
    from oracle import exact as X
    rng = np.random.default_rng(70 + M)
    _, W, T = S.uniform_batch(2, M, seed=71 + M)
    for b in range(2):
        ED = rng.normal(scale=0.3, size=(2, 3, 3)) if b == 1 else None
        J, dJ = X.refine_grad(W[b], T[b], ED)
        Tf = [Fraction(float(t)) for t in T[b]]
        assert sum(J) == X.optimal_cost(W[b], Tf, ED)
        for i in range(M):
            h = Tf[i] / 10 ** 25
            Tp, Tm = list(Tf), list(Tf)
            Tp[i] += h
            Tm[i] -= h
            fd = (X.optimal_cost(W[b], Tp, ED) - X.optimal_cost(W[b], Tm, ED)) / (2 * h)
            assert abs(fd - dJ[i]) <= Fraction(1, 10 ** 40) * (abs(dJ[i]) + 1)


def test_exact_cost_is_the_survey_hessian():
    """sum_i J_i of oracle/exact.py equals sum c^T Q c with the survey's a1 Hessian
    Q_jk = j!/(j-4)! k!/(k-4)! T^(j+k-7)/(j+k-7) on the exact coefficients, exactly."""
    from oracle import exact as X
    _, W, T = S.uniform_batch(1, 4, seed=77)
    ED = np.random.default_rng(77).normal(size=(2, 3, 3))
    C = X.reduced_solve(W[0], T[0], ED)
    J, _ = X.refine_grad(W[0], T[0], ED)
    q = Fraction(0)
    for i, t in enumerate(T[0]):
        Ti = Fraction(float(t))
        for a in range(3):
            c = C[i][a]
            for j in range(4, 8):
                for k in range(4, 8):
                    q += c[j] * c[k] * X.dfac(j, 4) * X.dfac(k, 4) * Ti ** (j + k - 7) / (j + k - 7)
    assert q == sum(J)


def test_gradient_recovery_is_exact_enough():
    """The GPU parity test recovers the applied gradient from T_1 (conftest.recovered_gradient).
    On the fixture's own exact T_1 (one rounding) that recovery is within 1e-11 of the exact
    gradient, so a 1e-9 bound on the GPU's recovered gradient measures the GPU."""
    k_T, eta, groups = load_refine_golden()
    for g, d in groups.items():
        rec, free = recovered_gradient(d["seg_times"], d["T1"], np.repeat(d["F"], np.diff(d["seg_offsets"])),
                                       k_T, eta)
        assert free.mean() > 0.9, g
        assert gradient_rel_err(d["seg_offsets"], rec, d["dJ"], free) <= 1e-11, g


@pytest.mark.parametrize("group", ["u10", "u10e", "u7e", "u16", "r", "re", "u257", "u257e", "r257", "r257e"])
def test_oracle_step_matches_exact_fixture(oracle, group):
    """The fp64 oracle's gradient (displacement form, the solve's own knot data) within 1e-9 of
    the exact dJ_i/dT_i, norm-wise per trajectory (measured <= 1e-10 on the small groups and
    8.2e-10 on r257e, where the dense Cholesky's ~2e-11 knot-data error is amplified ~30x; the
    round-5 form that re-evaluated the septic at T from absolute positions was 1e-9 off on 24
    trajectories already);
    F and one step's T_1 within 1e-11 (measured 1.3e-12 on F)."""
    k_T, eta, groups = load_refine_golden()
    d = groups[group]
    so, W, T, ED = d["seg_offsets"], d["waypoints"], d["seg_times"], d["end_derivs"]
    B = len(so) - 1
    dJ = np.zeros_like(T)
    Fo = np.zeros(B)
    for b in range(B):
        s0, s1 = int(so[b]), int(so[b + 1])
        g, Fo[b], st = oracle.refine_grad(W[s0 + b:s1 + b + 1], T[s0:s1], None if ED is None else ED[b], k_T,
                                          oracle.REDUCED)
        assert st == 0
        dJ[s0:s1] = g
    assert gradient_rel_err(so, dJ, d["dJ"]) <= 1e-9
    assert np.abs(Fo / d["F"] - 1).max() <= 1e-11
    T1, F0, _, st = oracle.refine_batch(so, W, T, ED, k_T, eta, 1, oracle.REDUCED)
    assert (st == 0).all()
    assert np.abs(T1 / d["T1"] - 1).max() <= 1e-11
