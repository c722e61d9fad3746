"""Generate the golden fixtures in tests/golden/ (run in the dev container only).

The reference repository has no min-snap solver, no tests and no fixtures
(SURVEY.md §0, §4), so these vectors come from EXACT rational arithmetic
(oracle/exact.py): every fp64 input is converted exactly to a Fraction, the
problem of SURVEY.md §8(a) is solved with no rounding, and the result is rounded
once to fp64.  For M <= 5 the generator also solves the survey's literal KKT
exactly and asserts the two rational solutions are identical.

    python tests/golden/make_golden.py [case ...]

Outputs (numpy .npz, no pickles): one file per case with
    seg_offsets int32 [B+1], waypoints [S+B,3], seg_times [S], end_derivs [B,18] (optional),
    coeffs [S,3,8] (exact, rounded), and for sampled cases dt, sample_offsets, samples [n,12].

refine_grad.npz (the config-5 step) holds ten groups, each
prefixed ``<g>_`` (u10, u10e: uniform M = 10 without / with end derivatives; u7e: M = 7
with; u16: M = 16; r, re: ragged M in 1..16, every M at least twice, without / with;
u257, u257e, r257, r257e: the 257-trajectory inputs of test_gpu_parity.py's one-step test):
    seg_offsets, waypoints, seg_times, end_derivs (the "e" groups),
    J [S], dJ [S]  exact per-segment snap cost and dJ_i/dT_i, rounded once,
    F [B]          exact F = sum J + k_T sum T, rounded once,
    T1 [S]         one step at (k_T, eta) = (REFINE_KT, REFINE_ETA): mpmath exp, rounded once.
"""
from __future__ import annotations

import os
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import exact as X  # noqa: E402
from trajectory_generator_ros2_amd import synthetic as S  # noqa: E402


def _csr(Ws, Ts):
    so = np.zeros(len(Ts) + 1, dtype=np.int32)
    so[1:] = np.cumsum([len(t) for t in Ts])
    return so, np.concatenate([np.asarray(w, float).reshape(-1, 3) for w in Ws]), np.concatenate(
        [np.asarray(t, float) for t in Ts])


def _solve_all(Ws, Ts, EDs=None, check_kkt_upto=5):
    out = []
    for i, (w, t) in enumerate(zip(Ws, Ts)):
        ed = None if EDs is None else np.asarray(EDs[i]).reshape(2, 3, 3)
        c = X.reduced_solve(w, t, ed)
        if len(t) <= check_kkt_upto:
            assert X.kkt_solve(w, t, ed) == c, "exact KKT and exact reduced solutions differ"
        out.append(np.vectorize(float)(np.array(c, dtype=object)).astype(np.float64))
    return np.concatenate(out, axis=0)


ONLY = set(sys.argv[1:])
REFINE_KT, REFINE_ETA = 1.0, 0.02


def _refine_one(args):
    w, t, ed = args
    J, dJ = X.refine_grad(w, t, None if ed is None else np.asarray(ed).reshape(2, 3, 3))
    Fv, T1 = X.refine_step(t, J, dJ, REFINE_KT, REFINE_ETA)
    return [float(v) for v in J], [float(v) for v in dJ], float(Fv), T1


def save_refine(groups):
    """groups: {name: (Ws, Ts, EDs or None)} -> refine_grad.npz (exact, parallel)."""
    if ONLY and "refine_grad" not in ONLY:
        return
    from multiprocessing import Pool
    d = dict(k_T=np.float64(REFINE_KT), eta=np.float64(REFINE_ETA))
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        for g, (Ws, Ts, EDs) in groups.items():
            so, W, T = _csr(Ws, Ts)
            res = pool.map(_refine_one, [(w, t, None if EDs is None else EDs[i]) for i, (w, t) in
                                         enumerate(zip(Ws, Ts))])
            d[g + "_seg_offsets"], d[g + "_waypoints"], d[g + "_seg_times"] = so, W, T
            if EDs is not None:
                d[g + "_end_derivs"] = np.asarray(EDs, float).reshape(-1, 18)
            d[g + "_J"] = np.concatenate([r[0] for r in res])
            d[g + "_dJ"] = np.concatenate([r[1] for r in res])
            d[g + "_F"] = np.asarray([r[2] for r in res])
            d[g + "_T1"] = np.concatenate([r[3] for r in res])
            print("refine_grad", g, "B=%d S=%d" % (len(Ts), int(so[-1])))
    np.savez_compressed(os.path.join(HERE, "refine_grad.npz"), **d)


def save(name, Ws, Ts, EDs=None, sample_dt=None):
    if ONLY and name not in ONLY:
        return
    so, W, T = _csr(Ws, Ts)
    C = _solve_all(Ws, Ts, EDs)
    d = dict(seg_offsets=so, waypoints=W, seg_times=T, coeffs=C)
    if EDs is not None:
        d["end_derivs"] = np.asarray(EDs, float).reshape(-1, 18)
    if sample_dt is not None:
        offs = [0]
        rows = []
        for i, (w, t) in enumerate(zip(Ws, Ts)):
            ed = None if EDs is None else np.asarray(EDs[i]).reshape(2, 3, 3)
            c = X.reduced_solve(w, t, ed)
            tot = 0.0
            for x in t:
                tot += float(x)
            n = int(np.ceil(tot / sample_dt - 1e-9))
            n = max(n, 1) + 1
            smp = X.sample_exact(c, t, w, ed, sample_dt, n)
            rows.extend([[float(v) for v in r] for r in smp])
            offs.append(offs[-1] + n)
        d["dt"] = np.float64(sample_dt)
        d["sample_offsets"] = np.asarray(offs, dtype=np.int64)
        d["samples"] = np.asarray(rows, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(name, "B=%d S=%d" % (len(Ts), int(so[-1])))


def main():
    rng = np.random.default_rng(7)
    # KAT: single rest-to-rest segment (closed form 35s^4-84s^5+70s^6-20s^7)
    _, W1, T1 = S.uniform_batch(8, 1, seed=11)
    save("kat_single", list(W1), list(T1))
    # config 1: B=1, M=3, the seed of SURVEY.md §8(d)
    _, Wc1, Tc1 = S.uniform_batch(1, 3)
    save("c1", list(Wc1), list(Tc1), sample_dt=0.01)
    # config 2 shape (M=3), small B
    _, W2, T2 = S.uniform_batch(64, 3, seed=S.SEED + 2)
    save("c2_small", list(W2), list(T2))
    # config 3 shape (M=10), small B
    _, W3, T3 = S.uniform_batch(16, 10, seed=S.SEED + 3)
    save("c3_small", list(W3), list(T3))
    save("c3_sampled", list(W3[:2]), list(T3[:2]), sample_dt=0.05)
    # ragged: every M in 1..16 at least once
    Ms = list(range(1, 17)) + list(rng.integers(2, 17, size=8))
    Wr, Tr = [], []
    for i, m in enumerate(Ms):
        _, w, t = S.uniform_batch(1, int(m), seed=1000 + i)
        Wr.append(w[0]); Tr.append(t[0])
    save("ragged", Wr, Tr)
    # non-rest end derivatives (braking / generateStopTraj path)
    _, We, Te = S.uniform_batch(16, 4, seed=S.SEED + 5)
    EDs = rng.normal(scale=[[[1.0], [0.5], [0.25]]] * np.ones((2, 3, 3)), size=(16, 2, 3, 3))
    save("end_derivs", list(We), list(Te), list(EDs), sample_dt=0.05)
    # extreme times (0.5 s next to 10 s), translated far from the origin, M=16
    Wx, Tx = [], []
    for i in range(4):
        _, w, t = S.uniform_batch(1, 16, seed=2000 + i)
        t = np.where(np.arange(16) % 2 == i % 2, 0.5, 10.0)
        Wx.append(w[0] + np.array([1000.0, -2000.0, 500.0]) * (i % 2)); Tx.append(t)
    save("extreme", Wx, Tx)
    # collinear waypoints: the solution must stay on the line
    Wl, Tl = [], []
    for i in range(4):
        a = rng.uniform(-5, 5, 3); d = rng.normal(size=3); d /= np.linalg.norm(d)
        s = np.sort(rng.uniform(-3, 3, 6))
        Wl.append(a + s[:, None] * d); Tl.append(rng.uniform(0.5, 3.0, 5))
    save("collinear", Wl, Tl)
    # config-5 refinement step: exact gradient and one exact step
    rr = np.random.default_rng(64)
    ed = lambda n: list(rr.normal(scale=0.3, size=(n, 18)))
    groups = {}
    for g, B, M, with_ed in (("u10", 32, 10, False), ("u10e", 32, 10, True), ("u7e", 16, 7, True),
                             ("u16", 16, 16, False)):
        _, Wu, Tu = S.uniform_batch(B, M, seed=3000 + M + 100 * with_ed)
        groups[g] = (list(Wu), list(Tu), ed(B) if with_ed else None)
    for g, with_ed in (("r", False), ("re", True)):
        Ms = list(range(1, 17)) * 2 + list(rr.integers(1, 17, size=8))
        Wr, Tr = [], []
        for i, m in enumerate(Ms):
            _, w, t = S.uniform_batch(1, int(m), seed=4000 + 100 * with_ed + i)
            Wr.append(w[0]); Tr.append(t[0])
        groups[g] = (Wr, Tr, ed(len(Ms)) if with_ed else None)
    # the one-step GPU test's own inputs (tests/test_gpu_parity.py): 257 trajectories each
    for ragged in (False, True):
        if ragged:
            so, W, T = S.ragged_batch(257, 1, 16, seed=61)
        else:
            so, W, T = S.uniform_batch(257, 10, seed=62)
        W, T = W.reshape(-1, 3), T.reshape(-1)
        Wl = [W[so[b] + b:so[b + 1] + b + 1] for b in range(257)]
        Tl = [T[so[b]:so[b + 1]] for b in range(257)]
        EDl = list(np.random.default_rng(63).normal(scale=0.3, size=(257, 18)))
        g = "r257" if ragged else "u257"
        groups[g] = (Wl, Tl, None)
        groups[g + "e"] = (Wl, Tl, EDl)
    save_refine(groups)


if __name__ == "__main__":
    main()
