"""Exact rational-arithmetic minimum-snap solves (TEST INFRASTRUCTURE ONLY).

Only ``tests/`` (and the golden-fixture generator ``tests/golden/make_golden.py``)
may import this module.  It is the strongest pin the oracle has: the reference
(jrached/trajectory_generator_ros2) contains no min-snap solver, tests or fixtures
(SURVEY.md §0, §4), so parity against it is UNPINNED; instead every fp64 input is
converted exactly to a ``Fraction`` and the problem of SURVEY.md §8(a) is solved
with no rounding at all.  Two formulations are provided:

* ``kkt_solve``      – the survey's literal C4 KKT system (rows a1–a3), Gaussian
                       elimination over the rationals (small M only: O(N^3) with
                       growing denominators);
* ``reduced_solve``  – the reduced system over the free knot derivatives
                       (v, a, j at interior knots), using the exactly derived
                       septic-Hermite snap-cost matrix.

For the time-allocation refinement:

* ``refine_grad``    – the exact per-segment snap cost J_i and its derivative
                       dJ_i/dT_i at the optimal knot data (envelope theorem), from
                       the definition sum_ab KH_ab T^(s_a+s_b-7) g_a g_b — no
                       displacement form, no rounding;
* ``optimal_cost``   – the exact optimal cost J*(T) = sum_i J_i, so a test can
                       check dJ_i/dT_i against an exact central difference of J*;
* ``refine_step``    – one step T_1 = T_0 exp(clamp(-eta T_0 (dJ + k_T) / F, +-1/2))
                       with F exact and exp in mpmath at 40 digits, rounded once.

For M <= 4 the tests require both to return *identical rationals*, which proves
the reduced formulation (the one the HIP kernel uses) is the same problem as the
KKT the north star names; the reduced solver then produces exact goldens up to
M = 16.
"""
from __future__ import annotations

from fractions import Fraction
from math import factorial
from typing import List, Optional, Sequence

F = Fraction


def dfac(j: int, k: int) -> int:
    """j!/(j-k)! (the k-th derivative factor of t^j); 0 when k > j."""
    return factorial(j) // factorial(j - k) if k <= j else 0


def _solve_exact(A: List[List[F]], B: List[List[F]]) -> List[List[F]]:
    """Gauss-Jordan over the rationals; A is n x n, B is n x r.  Raises on singular."""
    n = len(A)
    A = [row[:] for row in A]
    B = [row[:] for row in B]
    for k in range(n):
        p = next((i for i in range(k, n) if A[i][k] != 0), None)
        if p is None:
            raise ZeroDivisionError("singular system")
        A[k], A[p] = A[p], A[k]
        B[k], B[p] = B[p], B[k]
        inv = 1 / A[k][k]
        rowk = A[k]
        bk = B[k]
        for i in range(n):
            if i == k or A[i][k] == 0:
                continue
            f = A[i][k] * inv
            rowi = A[i]
            for j in range(k, n):
                if rowk[j]:
                    rowi[j] -= f * rowk[j]
            bi = B[i]
            for r in range(len(bi)):
                bi[r] -= f * bk[r]
    return [[B[i][r] / A[i][i] for r in range(len(B[i]))] for i in range(n)]


def hermite_maps():
    """Exact septic-Hermite maps on s in [0,1].

    Returns (E, KH): E (8x8) maps scaled end data h = [y0,y0',y0'',y0''',y1,y1',y1'',y1''']
    to monomial coefficients d; KH = E^T H4 E is the snap-cost matrix,
    integral_0^1 (q'''')^2 ds = h^T KH h.
    """
    # constraint matrix: row (end e, derivative k), column monomial j
    S = []
    for e in (0, 1):
        for k in range(4):
            S.append([F(dfac(j, k)) * (F(e) ** (j - k) if j >= k else 0) for j in range(8)])
    # reorder rows to h ordering [start k=0..3, end k=0..3] (already in that order)
    I8 = [[F(int(i == j)) for j in range(8)] for i in range(8)]
    E = _solve_exact(S, I8)  # d = E h
    H4 = [[F(dfac(j, 4) * dfac(k, 4), j + k - 7) if (j >= 4 and k >= 4) else F(0) for k in range(8)]
          for j in range(8)]
    EtH = [[sum(E[a][j] * H4[a][k] for a in range(8)) for k in range(8)] for j in range(8)]
    KH = [[sum(EtH[x][k] * E[k][y] for k in range(8)) for y in range(8)] for x in range(8)]
    return E, KH


_E, _KH = hermite_maps()
_SIG = [0, 1, 2, 3, 0, 1, 2, 3]


def _as_frac_traj(waypoints, seg_times, end_derivs):
    M = len(seg_times)
    W = [[F(float(waypoints[i][a])) for a in range(3)] for i in range(M + 1)]
    T = [F(float(t)) for t in seg_times]
    if end_derivs is None:
        ED = [[[F(0)] * 3 for _ in range(3)] for _ in range(2)]
    else:
        ED = [[[F(float(end_derivs[e][k][a])) for a in range(3)] for k in range(3)] for e in range(2)]
    return M, W, T, ED


def kkt_solve(waypoints, seg_times, end_derivs=None, cont: int = 4):
    """Exact solve of the survey's KKT (a1–a3).  Returns coeffs[M][3][8] as Fractions."""
    M, W, T, ED = _as_frac_traj(waypoints, seg_times, end_derivs)
    n = 8 * M
    rows = []  # (dict col->val, rhs[3])

    def drow(k, t):
        return [F(dfac(j, k)) * (t ** (j - k)) if j >= k else F(0) for j in range(8)]

    for k in range(4):
        rows.append(({j: v for j, v in enumerate(drow(k, F(0)))}, W[0] if k == 0 else ED[0][k - 1]))
    for k in range(4):
        r = drow(k, T[M - 1])
        rows.append(({8 * (M - 1) + j: v for j, v in enumerate(r)}, W[M] if k == 0 else ED[1][k - 1]))
    zero = [F(0)] * 3
    for i in range(1, M):
        rows.append(({8 * (i - 1) + j: v for j, v in enumerate(drow(0, T[i - 1]))}, W[i]))
        rows.append(({8 * i + j: v for j, v in enumerate(drow(0, F(0)))}, W[i]))
        for k in range(1, cont + 1):
            d = {8 * (i - 1) + j: v for j, v in enumerate(drow(k, T[i - 1]))}
            for j, v in enumerate(drow(k, F(0))):
                d[8 * i + j] = d.get(8 * i + j, F(0)) - v
            rows.append((d, zero))
    m = len(rows)
    N = n + m
    K = [[F(0)] * N for _ in range(N)]
    R = [[F(0)] * 3 for _ in range(N)]
    for i in range(M):
        for j in range(4, 8):
            for k in range(4, 8):
                e = j + k - 7
                K[8 * i + j][8 * i + k] = 2 * F(dfac(j, 4) * dfac(k, 4), e) * T[i] ** e
    for r, (d, b) in enumerate(rows):
        for c, v in d.items():
            if v:
                K[n + r][c] += v
                K[c][n + r] += v
        R[n + r] = list(b)
    X = _solve_exact(K, R)
    return [[[X[8 * i + j][a] for j in range(8)] for a in range(3)] for i in range(M)]


def reduced_solve(waypoints, seg_times, end_derivs=None):
    """Exact solve through the reduced Hessian over free knot derivatives."""
    return _reduced(*_as_frac_traj(waypoints, seg_times, end_derivs))[0]


def _reduced(M, W, T, ED):
    """Exact reduced solve: (coeffs[M][3][8], knot data kd(knot, axis) -> [p, v, a, j])."""
    nf = 3 * (M - 1)

    def known(knot, d, a):
        if d == 0:
            return W[knot][a]
        return ED[0 if knot == 0 else 1][d - 1][a]

    U = None
    if nf:
        H = [[F(0)] * nf for _ in range(nf)]
        R = [[F(0)] * 3 for _ in range(nf)]
        for i in range(M):
            Ks = [[_KH[x][y] * T[i] ** (_SIG[x] + _SIG[y] - 7) for y in range(8)] for x in range(8)]
            for x in range(8):
                kx, dx = (i if x < 4 else i + 1), x & 3
                if dx == 0 or kx in (0, M):
                    continue
                rx = 3 * (kx - 1) + dx - 1
                for y in range(8):
                    ky, dy = (i if y < 4 else i + 1), y & 3
                    if dy != 0 and ky not in (0, M):
                        H[rx][3 * (ky - 1) + dy - 1] += Ks[x][y]
                    else:
                        for a in range(3):
                            R[rx][a] -= Ks[x][y] * known(ky, dy, a)
        U = _solve_exact(H, R)

    def kd(knot, a):
        out = [W[knot][a]]
        for d in (1, 2, 3):
            if knot in (0, M):
                out.append(known(knot, d, a))
            else:
                out.append(U[3 * (knot - 1) + d - 1][a])
        return out

    C = []
    for i in range(M):
        seg = []
        for a in range(3):
            g0, g1 = kd(i, a), kd(i + 1, a)
            h = [g0[q] * T[i] ** _SIG[q] for q in range(4)] + [g1[q] * T[i] ** _SIG[q] for q in range(4)]
            d = [sum(_E[j][q] * h[q] for q in range(8)) for j in range(8)]
            seg.append([d[j] / T[i] ** j for j in range(8)])
        C.append(seg)
    return C, kd


def _segment_cost(T: F, g0, g1):
    """J and dJ/dT of one axis of one segment from its end data, by definition."""
    g = list(g0) + list(g1)
    j = dj = F(0)
    for x in range(8):
        for y in range(8):
            n = _SIG[x] + _SIG[y] - 7
            k = _KH[x][y] * g[x] * g[y]
            j += k * T ** n
            dj += k * n * T ** (n - 1)
    return j, dj


def refine_grad(waypoints, seg_times, end_derivs=None):
    """Exact per-segment snap cost J_i and dJ_i/dT_i (knot data held at the optimum)."""
    M, W, T, ED = _as_frac_traj(waypoints, seg_times, end_derivs)
    _, kd = _reduced(M, W, T, ED)
    J, dJ = [], []
    for i in range(M):
        ji = dji = F(0)
        for a in range(3):
            j, dj = _segment_cost(T[i], kd(i, a), kd(i + 1, a))
            ji += j
            dji += dj
        J.append(ji)
        dJ.append(dji)
    return J, dJ


def optimal_cost(waypoints, seg_times, end_derivs=None):
    """Exact optimal snap cost J*(T) for times given as Fractions or floats."""
    M = len(seg_times)
    W = [[F(float(waypoints[i][a])) for a in range(3)] for i in range(M + 1)]
    T = [t if isinstance(t, F) else F(float(t)) for t in seg_times]
    if end_derivs is None:
        ED = [[[F(0)] * 3 for _ in range(3)] for _ in range(2)]
    else:
        ED = [[[F(float(end_derivs[e][k][a])) for a in range(3)] for k in range(3)] for e in range(2)]
    _, kd = _reduced(M, W, T, ED)
    return sum(_segment_cost(T[i], kd(i, a), kd(i + 1, a))[0] for i in range(M) for a in range(3))


def refine_step(seg_times, J, dJ, k_T: float, eta: float):
    """One refinement step from exact J_i, dJ_i: returns (F, T_1 as floats).

    F = sum J_i + k_T sum T_i (exact), dtau_i = clamp(-eta T_i (dJ_i + k_T) / F, -1/2, 1/2)
    (exact), T_1 = T_i exp(dtau_i) in mpmath at 40 significant digits, rounded to fp64 once.
    The step is csrc/tgms_reduced.hip's and oracle_refine_times' (SURVEY.md §8(f) rank 2)."""
    import mpmath
    T = [F(float(t)) for t in seg_times]
    kT, et = F(float(k_T)), F(float(eta))
    Fv = sum(J) + kT * sum(T)
    half = F(1, 2)
    out = []
    with mpmath.workdps(40):
        for Ti, g in zip(T, dJ):
            d = -et * Ti * (g + kT) / Fv
            d = min(max(d, -half), half)
            x = mpmath.mpf(Ti.numerator) / Ti.denominator * mpmath.exp(mpmath.mpf(d.numerator) / d.denominator)
            out.append(float(x))
    return Fv, out


def eval_exact(coeffs_seg_axis: Sequence[F], t: F, k: int) -> F:
    """k-th derivative of one septic at local time t, exactly."""
    return sum(F(dfac(j, k)) * coeffs_seg_axis[j] * t ** (j - k) for j in range(k, 8))


def sample_exact(coeffs, seg_times, waypoints, end_derivs, dt: float, n: int):
    """Exact p/v/a/j at t_k = k*dt (fp64 products rounded as the kernel computes
    them, i.e. t = float(k) * dt in fp64), k = 0..n-2, plus the pinned final sample.
    Returns rows of 12 Fractions (p, v, a, j) — yaw is checked separately."""
    M = len(seg_times)
    tau = [0.0]
    for t in seg_times:
        tau.append(tau[-1] + float(t))  # fp64 accumulation, as the kernel and oracle do
    out = []
    for k in range(n - 1):
        t = float(k) * dt
        i = 0
        while i + 1 < M and tau[i + 1] <= t:
            i += 1
        lt = F(t - tau[i])  # fp64 subtraction, then exact evaluation
        row = []
        for d in range(4):
            for a in range(3):
                row.append(eval_exact(coeffs[i][a], lt, d))
        out.append(row)
    last = [F(float(waypoints[M][a])) for a in range(3)]
    for d in range(3):
        for a in range(3):
            last.append(F(0) if end_derivs is None else F(float(end_derivs[1][d][a])))
    out.append(last)
    return out


def closed_form_single(w0: float, w1: float, T: float, t: float) -> F:
    """Rest-to-rest single segment: p(t) = w0 + (w1-w0)(35s^4 - 84s^5 + 70s^6 - 20s^7), s = t/T."""
    s = F(t) / F(T)
    return F(w0) + (F(w1) - F(w0)) * (35 * s ** 4 - 84 * s ** 5 + 70 * s ** 6 - 20 * s ** 7)
