"""CPU: pin the oracle (the checker of every GPU parity test).

The reference has no min-snap solver, tests or fixtures, so the
oracle is pinned by exact rational arithmetic instead:
  * the survey's literal KKT (a1-a3) and the reduced system solved EXACTLY give
    identical rationals (so the HIP kernel's formulation is the same problem);
  * the fp64 oracle matches the exact goldens in tests/golden/ to 1e-12;
  * closed-form single-segment KAT, linearity, translation, time reversal,
    collinearity and C6 smoothness.
"""
import os

import numpy as np
import pytest

from conftest import batch_rel_err, solve_goldens

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLDENS = solve_goldens()
ORACLE_TOL = 1e-12   # dense KKT / square C6 oracle vs exact
REDUCED_TOL = 1e-10  # reduced-Hessian restatement: knot derivatives -> monomials amplifies rounding


def _traj(g, b):
    so = g["seg_offsets"]
    s0, s1 = int(so[b]), int(so[b + 1])
    ED = g["end_derivs"][b].reshape(2, 3, 3) if "end_derivs" in g.files else None
    return g["waypoints"][s0 + b:s1 + b + 1], g["seg_times"][s0:s1], ED, g["coeffs"][s0:s1]


@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_exact_kkt_equals_exact_reduced(M):
    from oracle import exact as X
    from trajectory_generator_ros2_amd import synthetic as S
    rng = np.random.default_rng(M)
    _, W, T = S.uniform_batch(2, M, seed=50 + M)
    for b in range(2):
        ED = rng.normal(size=(2, 3, 3)) if b else None
        assert X.kkt_solve(W[b], T[b], ED) == X.reduced_solve(W[b], T[b], ED)


def test_exact_kkt_c3_equals_c4():
    from oracle import exact as X
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(1, 3, seed=77)
    assert X.kkt_solve(W[0], T[0], cont=3) == X.kkt_solve(W[0], T[0], cont=4)


def test_hermite_cost_matrix_is_integer_and_psd():
    from oracle import exact as X
    _, KH = X.hermite_maps()
    assert all(v.denominator == 1 for row in KH for v in row)
    K = np.array([[float(v) for v in row] for row in KH])
    assert np.allclose(K, K.T)
    ev = np.linalg.eigvalsh(K)
    assert ev.min() > -1e-6 * ev.max() and np.sum(ev > 1e-6 * ev.max()) == 4  # rank 4


@pytest.mark.parametrize("path", GOLDENS, ids=[os.path.basename(p) for p in GOLDENS])
@pytest.mark.parametrize("form", [0, 1, 2, 3, 4], ids=["kkt_c4", "kkt_c3", "square_c6", "reduced", "kkt_band"])
def test_oracle_vs_exact_goldens(oracle, path, form):
    g = np.load(path)
    so = g["seg_offsets"]
    ED = g["end_derivs"] if "end_derivs" in g.files else None
    C, st = oracle.solve_batch(so, g["waypoints"], g["seg_times"], ED, form)
    assert (st == 0).all()
    assert batch_rel_err(so, C, g["coeffs"]) <= (REDUCED_TOL if form == 3 else ORACLE_TOL)


def test_kat_single_segment_closed_form(oracle):
    from oracle import exact as X
    g = np.load(os.path.join(GOLDEN, "kat_single.npz"))
    for b in range(len(g["seg_offsets"]) - 1):
        W, T, _, Cx = _traj(g, b)
        for t in np.linspace(0.0, T[0], 7):
            for a in range(3):
                ref = float(X.closed_form_single(W[0, a], W[1, a], T[0], t))
                got = np.polyval(Cx[0, a, ::-1], t)
                assert abs(got - ref) <= 1e-12 * (1 + abs(ref))


@pytest.mark.parametrize("M", [1, 2, 3, 10, 16])
def test_interleaved_kkt_is_banded(oracle, M):
    """The order TGMS_METHOD_BAND_KKT eliminates in ([start | c_0 | knot 1 | c_1 | ... |
    end]) puts every nonzero of the KKT within 9 of the diagonal, so GEPP keeps L in
    9 sub-diagonals and U in 18 super-diagonals: the band kernel skips only zeros."""
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(1, M, seed=M)
    K, _ = oracle.assemble_kkt(W[0], T[0])
    n = 8 * M
    order = list(range(n, n + 4))
    for i in range(M):
        order += list(range(8 * i, 8 * i + 8))
        if i < M - 1:
            order += list(range(n + 8 + 6 * i, n + 14 + 6 * i))
    order += list(range(n + 4, n + 8))
    assert sorted(order) == list(range(14 * M + 2))
    P = K[np.ix_(order, order)]
    r, c = np.nonzero(P)
    assert np.abs(r - c).max() <= 9
    # GEPP on the permuted matrix: no fill outside the band
    A = P.copy()
    N = A.shape[0]
    for k in range(N):
        p = k + int(np.argmax(np.abs(A[k:, k])))
        A[[k, p]] = A[[p, k]]
        A[k + 1:, k] /= A[k, k]
        A[k + 1:, k + 1:] -= np.outer(A[k + 1:, k], A[k, k + 1:])
        assert not A[k + 10:, k].any()
    assert not np.triu(A, 19).any()


def test_kkt_assembly_structure(oracle):
    """a1/a2 shapes and the block structure of [[2Q, A^T],[A, 0]]."""
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(1, 10)
    K, rhs = oracle.assemble_kkt(W[0], T[0])
    n, N = 80, 142
    assert K.shape == (N, N) and rhs.shape == (N, 3)
    assert np.array_equal(K, K.T)
    assert not K[n:, n:].any()                  # zero multiplier block
    assert not rhs[:n].any()                    # [0; b]
    Q = K[:n, :n]
    for i in range(10):                          # block-diagonal, only powers 4..7 nonzero
        blk = Q[8 * i:8 * i + 8, 8 * i:8 * i + 8]
        assert not blk[:4].any() and not blk[:, :4].any()
        assert np.all(np.linalg.eigvalsh(blk[4:, 4:]) > 0)
    off = Q.copy()
    for i in range(10):
        off[8 * i:8 * i + 8, 8 * i:8 * i + 8] = 0
    assert not off.any()
    assert np.linalg.matrix_rank(K[n:, :n]) == N - n   # A has full row rank


def test_properties(oracle):
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(4, 7, seed=3)
    for b in range(4):
        C, _ = oracle.solve(W[b], T[b])
        # linearity: c(alpha W) = alpha c(W)
        C2, _ = oracle.solve(2.5 * W[b], T[b])
        assert np.abs(C2 - 2.5 * C).max() <= 1e-12 * np.abs(C).max() * 2.5
        # translation: adding a constant shifts only c0
        sh = np.array([3.0, -7.0, 11.0])
        C3, _ = oracle.solve(W[b] + sh, T[b])
        d = C3 - C
        assert np.abs(d[:, :, 0] - sh).max() <= 1e-12 * 20
        assert np.abs(d[:, :, 1:]).max() <= 1e-11 * np.abs(C).max()
        # time reversal: reversed waypoints/times give p(T - t)
        Cr, _ = oracle.solve(W[b][::-1].copy(), T[b][::-1].copy())
        for i in range(7):
            ir = 6 - i
            for t in np.linspace(0, T[b][i], 5):
                p = np.polyval(C[i, :, ::-1].T, t) if False else [np.polyval(C[i, a, ::-1], t) for a in range(3)]
                q = [np.polyval(Cr[ir, a, ::-1], T[b][i] - t) for a in range(3)]
                assert np.abs(np.array(p) - np.array(q)).max() <= 1e-10


def test_collinear_stays_on_line(oracle):
    g = np.load(os.path.join(GOLDEN, "collinear.npz"))
    for b in range(len(g["seg_offsets"]) - 1):
        W, T, _, _ = _traj(g, b)
        C, _ = oracle.solve(W, T)
        d = W[-1] - W[0]
        d /= np.linalg.norm(d)
        for i in range(len(T)):
            for t in np.linspace(0, T[i], 9):
                p = np.array([np.polyval(C[i, a, ::-1], t) for a in range(3)]) - W[0]
                assert np.linalg.norm(p - d * (p @ d)) <= 1e-9


def test_c6_smoothness(oracle):
    """The minimiser is a C6 septic spline although only C4 is constrained."""
    from math import factorial
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(3, 9, seed=8)
    for b in range(3):
        C, _ = oracle.solve(W[b], T[b])
        for i in range(8):
            for k in range(1, 7):
                left = sum(factorial(j) / factorial(j - k) * C[i, :, j] * T[b][i] ** (j - k) for j in range(k, 8))
                right = factorial(k) * C[i + 1, :, k]
                assert np.abs(left - right).max() <= 1e-8 * (1 + np.abs(right).max())


def test_invalid_inputs(oracle):
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(1, 3)
    T = T[0].copy()
    T[1] = 0.0
    assert oracle.solve(W[0], T)[1] == 1
    T[1] = np.nan
    assert oracle.solve(W[0], T)[1] == 1
    W2 = W[0].copy()
    W2[2, 0] = np.inf
    assert oracle.solve(W2, np.ones(3))[1] == 1


@pytest.mark.parametrize("name", ["c1", "c3_sampled", "end_derivs"])
def test_oracle_sampler_vs_exact(oracle, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    offs = g["sample_offsets"]
    dt = float(g["dt"])
    for b in range(len(g["seg_offsets"]) - 1):
        W, T, ED, Cx = _traj(g, b)
        out = oracle.sample(Cx, T, W, ED, dt)
        ref = g["samples"][offs[b]:offs[b + 1]]
        assert out.shape[0] == ref.shape[0]
        for f0, f1 in ((0, 3), (3, 6), (6, 9), (9, 12)):
            sc = np.abs(ref[:, f0:f1]).max()
            assert np.abs(out[:, f0:f1] - ref[:, f0:f1]).max() <= 1e-12 * max(sc, 1.0)
        assert np.array_equal(out[-1, :3], W[-1])   # last sample pinned to the final waypoint


def test_sample_count_convention(oracle):
    assert oracle.sample_count(1.0, 0.01) == 101   # t = 0 .. 0.99 plus the pinned t = 1.0
    assert oracle.sample_count(0.005, 0.01) == 2
    assert oracle.sample_count(0.0, 0.01) == 2
    assert oracle.sample_count(10.0, 0.1) == 101


def test_spline_property_checker(oracle):
    """conftest.check_spline_properties (used at full size on the GPU) accepts the
    oracle's solution of a ragged batch and rejects a perturbed one."""
    from conftest import check_spline_properties
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(200, 1, 16, seed=3)
    C, st = oracle.solve_batch(so, W, T, None, oracle.REDUCED)
    assert (st == 0).all()
    check_spline_properties(so, W, T, C)
    bad = C.copy()
    bad[int(so[7]) + 1, 2, 5] += 1e-3  # a kink inside trajectory 7 (M >= 2 there?)
    if so[8] - so[7] < 2:
        bad[int(so[8]) - 1, 2, 5] += 1e-3
    with pytest.raises(AssertionError):
        check_spline_properties(so, W, T, bad)
