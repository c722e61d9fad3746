"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Importable only from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, as the checker / the timed CPU baseline — never from the
product package ``trajectory_generator_ros2_amd``.  See ``minsnap_oracle.h`` for
the formulation and for why parity against the reference is unpinned (the
reference has no min-snap solver), and ``exact.py`` for the rational pin.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

KKT_C4, KKT_C3, SQUARE_C6, REDUCED, KKT_BAND = 0, 1, 2, 3, 4
YAW_CONSTANT, YAW_VELOCITY = 0, 1

_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc, no reference sources)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        L.oracle_solve.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp]
        L.oracle_solve.restype = ctypes.c_int
        L.oracle_solve_batch.argtypes = [ctypes.c_int, ctypes.c_int32, ip, dp, dp, dp, dp, ip, ctypes.c_int]
        L.oracle_solve_batch.restype = ctypes.c_int
        L.oracle_assemble_kkt.argtypes = [ctypes.c_int, dp, dp, dp, dp, dp]
        L.oracle_assemble_kkt.restype = ctypes.c_int
        L.oracle_sample_count.argtypes = [ctypes.c_double, ctypes.c_double]
        L.oracle_sample_count.restype = ctypes.c_int64
        L.oracle_sample.argtypes = [ctypes.c_int, dp, dp, dp, dp, ctypes.c_double, ctypes.c_int,
                                    ctypes.c_double, dp]
        L.oracle_sample.restype = ctypes.c_int64
        L.oracle_refine_times.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, ctypes.c_double, ctypes.c_double,
                                          ctypes.c_int, dp, dp]
        L.oracle_refine_times.restype = ctypes.c_int
        L.oracle_refine_batch.argtypes = [ctypes.c_int, ctypes.c_int32, ip, dp, dp, dp, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_int, dp, dp, ip, ctypes.c_int]
        L.oracle_refine_batch.restype = ctypes.c_int
        L.oracle_refine_grad.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, ctypes.c_double, dp, dp]
        L.oracle_refine_grad.restype = ctypes.c_int
        _lib = L
    return _lib


def _dp(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def solve(waypoints, seg_times, end_derivs=None, formulation: int = KKT_C4):
    """One trajectory: waypoints (M+1,3), seg_times (M,), end_derivs (2,3,3) or None.
    Returns (coeffs (M,3,8), status)."""
    W = np.ascontiguousarray(waypoints, dtype=np.float64)
    T = np.ascontiguousarray(seg_times, dtype=np.float64)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64)
    M = T.shape[0]
    C = np.zeros((M, 3, 8), dtype=np.float64)
    st = lib().oracle_solve(formulation, M, _dp(W), _dp(T), _dp(ED), _dp(C))
    return C, st


def solve_batch(seg_offsets, waypoints, seg_times, end_derivs=None, formulation: int = KKT_C4,
                nthreads: int = 0):
    """CSR batch (the C-ABI layout).  Returns (coeffs [S,3,8], status [B])."""
    so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
    W = np.ascontiguousarray(waypoints, dtype=np.float64).reshape(-1, 3)
    T = np.ascontiguousarray(seg_times, dtype=np.float64).reshape(-1)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64).reshape(-1, 18)
    B = so.shape[0] - 1
    C = np.zeros((int(so[-1]), 3, 8), dtype=np.float64)
    st = np.zeros(B, dtype=np.int32)
    lib().oracle_solve_batch(formulation, B, _ip(so), _dp(W), _dp(T), _dp(ED), _dp(C), _ip(st), nthreads)
    return C, st


def assemble_kkt(waypoints, seg_times, end_derivs=None):
    W = np.ascontiguousarray(waypoints, dtype=np.float64)
    T = np.ascontiguousarray(seg_times, dtype=np.float64)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64)
    M = T.shape[0]
    N = 14 * M + 2
    K = np.zeros((N, N))
    rhs = np.zeros((N, 3))
    n = lib().oracle_assemble_kkt(M, _dp(W), _dp(T), _dp(ED), _dp(K), _dp(rhs))
    assert n == N, n
    return K, rhs


def sample_count(total_T: float, dt: float) -> int:
    return int(lib().oracle_sample_count(total_T, dt))


def sample(coeffs, seg_times, waypoints, end_derivs, dt, yaw_mode=YAW_CONSTANT, yaw_const=0.0):
    C = np.ascontiguousarray(coeffs, dtype=np.float64)
    T = np.ascontiguousarray(seg_times, dtype=np.float64)
    W = np.ascontiguousarray(waypoints, dtype=np.float64)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64)
    M = T.shape[0]
    n = sample_count(float(np.sum(T)), dt)  # same order of summation as the C code for M small
    out = np.zeros((n + 1, 14))
    got = lib().oracle_sample(M, _dp(C), _dp(T), _dp(W), _dp(ED), dt, yaw_mode, yaw_const, _dp(out))
    return out[:got]


def refine_times(waypoints, seg_times, end_derivs=None, k_T=1.0, eta=0.1, iters=10, formulation: int = KKT_C4):
    """One trajectory: (refined T, final cost F, final coefficients, status)."""
    W = np.ascontiguousarray(waypoints, dtype=np.float64)
    T = np.array(seg_times, dtype=np.float64)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64)
    M = T.shape[0]
    C = np.zeros((M, 3, 8))
    cost = np.zeros(1)
    st = lib().oracle_refine_times(formulation, M, _dp(W), _dp(T), _dp(ED), float(k_T), float(eta), int(iters),
                                   _dp(cost), _dp(C))
    return T, float(cost[0]), C, st


def refine_grad(waypoints, seg_times, end_derivs=None, k_T=1.0, formulation: int = REDUCED):
    """One trajectory at fixed times: (dJ_i/dT_i [M], F = sum J + k_T sum T, status) — the
    ingredients of one refinement step (oracle_refine_grad)."""
    W = np.ascontiguousarray(waypoints, dtype=np.float64)
    T = np.ascontiguousarray(seg_times, dtype=np.float64)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64)
    dJ = np.zeros(T.shape[0])
    cost = np.zeros(1)
    st = lib().oracle_refine_grad(formulation, T.shape[0], _dp(W), _dp(T), _dp(ED), float(k_T), _dp(dJ), _dp(cost))
    return dJ, float(cost[0]), st


def refine_batch(seg_offsets, waypoints, seg_times, end_derivs=None, k_T=1.0, eta=0.1, iters=10,
                 formulation: int = KKT_C4, nthreads: int = 0):
    """CSR batch: (refined T [S], cost [B], coeffs [S,3,8], status [B])."""
    so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
    W = np.ascontiguousarray(waypoints, dtype=np.float64).reshape(-1, 3)
    T = np.array(seg_times, dtype=np.float64).reshape(-1)
    ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64).reshape(-1, 18)
    B = so.shape[0] - 1
    C = np.zeros((int(so[-1]), 3, 8))
    cost = np.zeros(B)
    st = np.zeros(B, dtype=np.int32)
    lib().oracle_refine_batch(formulation, B, _ip(so), _dp(W), _dp(T), _dp(ED), float(k_T), float(eta), int(iters),
                              _dp(cost), _dp(C), _ip(st), nthreads)
    return T, cost, C, st

