#!/usr/bin/env python3
"""Coefficients of exp_step (csrc/tgms_reduced.hip): exp(x) on the refinement update's clamped
range |x| <= 0.5 as one degree-N polynomial, Horner with FMAs (no range reduction, no ldexp).

The coefficients interpolate exp at the N + 1 Chebyshev nodes of [-0.5, 0.5] (near-minimax),
computed at 60 digits with mpmath and rounded to double.  The check evaluates the double
Horner chain with every FMA rounded once (emulated exactly) at 20,001 points against
mpmath's exp, and reports the worst error in units of the last place of the true value.
  python3 scripts/exp_poly.py [N]"""
import sys
import mpmath as mp

mp.mp.dps = 60
N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
H = mp.mpf("0.5")
nodes = [H * mp.cos(mp.pi * (2 * k + 1) / (2 * (N + 1))) for k in range(N + 1)]
# monomial coefficients of the interpolant: solve the Vandermonde system at 60 digits
V = mp.matrix([[x ** j for j in range(N + 1)] for x in nodes])
y = mp.matrix([mp.exp(x) for x in nodes])
c = mp.lu_solve(V, y)
cd = [float(c[j]) for j in range(N + 1)]


def fma(a, b, s):  # one rounding, as v_fma_f64
    return float(mp.mpf(a) * mp.mpf(b) + mp.mpf(s))


def horner(x):
    p = cd[N]
    for j in range(N - 1, -1, -1):
        p = fma(p, x, cd[j])
    return p


worst = 0.0
for i in range(20001):
    x = float(-0.5 + mp.mpf(i) / 20000)
    t = mp.exp(mp.mpf(x))
    ulp = mp.mpf(2) ** (mp.floor(mp.log(t, 2)) - 52)
    worst = max(worst, float(abs(horner(x) - t) / ulp))
print("degree %d, worst error %.3f ulp over [-0.5, 0.5]" % (N, worst))
for j, v in enumerate(cd):
    print("    %s,  // x^%d" % (repr(v), j))
