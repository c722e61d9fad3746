"""Python front-end over the C ABI (numpy host buffers or torch device tensors).

Mirrors the reference's generate-then-consume flow: a batch of
waypoint sets goes in, order-7 coefficients [seg][axis][8] come out, and the
sampler turns them into Goal-like records at dt.  All compute runs in libtgms
(HIP); this module only marshals pointers.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import TgmsError


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags.c_contiguous, "arrays must be C-contiguous"
        return a.ctypes.data
    # torch tensor (device or host)
    assert a.is_contiguous(), "tensors must be contiguous"
    return a.data_ptr()


class Solver:
    """A libtgms handle bound to one HIP device (or, asked for explicitly, the host backend)."""

    def __init__(self, device: int = 0, method: int = _lib.METHOD_REDUCED, device_count: int = 0,
                 host: bool = False):
        """device_count > 0: a multi-GPU handle over devices 0..device_count-1
        (tgms_create_multi: one RCCL communicator per device); host=True: the explicit host
        backend (tgms_create_host: solve + sample on the CPU, config 1); else one device."""
        self._L = _lib.load()
        h = ctypes.c_void_p()
        if host:
            st = self._L.tgms_create_host(ctypes.byref(h))
            what = "tgms_create_host"
        elif device_count > 0:
            st = self._L.tgms_create_multi(ctypes.byref(h), int(device_count))
            what = "tgms_create_multi"
        else:
            st = self._L.tgms_create(ctypes.byref(h), int(device))
            what = "tgms_create"
        if st != _lib.OK:
            raise TgmsError(st, f"{what} failed (no CPU fallback exists)")
        self._h = h
        self.device = 0 if device_count > 0 else device
        self.device_count = int(self._L.tgms_device_count(h))
        self.set_method(method)

    def close(self):
        if getattr(self, "_h", None):
            self._L.tgms_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def last_error(self) -> str:
        return self._L.tgms_last_error(self._h).decode()

    def set_method(self, method: int):
        st = self._L.tgms_set_method(self._h, int(method))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())
        self.method = method

    # ---------------------------------------------------------------- host API
    def solve(self, seg_offsets, waypoints, seg_times, end_derivs=None, check: bool = True,
              out: Optional[Tuple[np.ndarray, np.ndarray]] = None) -> Tuple[np.ndarray, np.ndarray, int]:
        """CSR host batch -> (coeffs [S,3,8], status [B], worst status).

        `out` = (coeffs, status) reuses caller buffers (float64 [S,3,8], int32 [>=B]):
        fresh host pages fault in during the device-to-host copy, reused ones do not."""
        so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
        W = np.ascontiguousarray(waypoints, dtype=np.float64).reshape(-1, 3)
        T = np.ascontiguousarray(seg_times, dtype=np.float64).reshape(-1)
        ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64).reshape(-1, 18)
        B = so.shape[0] - 1
        S = int(so[-1]) if B > 0 else 0
        if out is not None:
            C, st = out
            if C.dtype != np.float64 or C.size < S * 24 or not C.flags.c_contiguous:
                raise ValueError("out coeffs must be C-contiguous float64 with >= S*24 elements")
            if st.dtype != np.int32 or st.size < max(B, 1) or not st.flags.c_contiguous:
                raise ValueError("out status must be C-contiguous int32 with >= B elements")
        else:
            C = np.zeros((S, 3, 8), dtype=np.float64)
            st = np.zeros(max(B, 1), dtype=np.int32)
        worst = self._L.tgms_solve_batch(self._h, B, _ptr(so), _ptr(W), _ptr(T), _ptr(ED), _ptr(C), _ptr(st))
        if check and worst not in (_lib.OK,) and worst in (_lib.ERR_DEVICE, _lib.ERR_NO_DEVICE):
            raise TgmsError(worst, self.last_error())
        return C, st[:B], worst

    def solve_multi(self, seg_offsets, waypoints, seg_times, end_derivs=None) -> Tuple[np.ndarray, np.ndarray, int]:
        """tgms_solve_batch_multi: host batch over every device of the handle."""
        so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
        W = np.ascontiguousarray(waypoints, dtype=np.float64).reshape(-1, 3)
        T = np.ascontiguousarray(seg_times, dtype=np.float64).reshape(-1)
        ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64).reshape(-1, 18)
        B = so.shape[0] - 1
        C = np.zeros((int(so[-1]) if B > 0 else 0, 3, 8), dtype=np.float64)
        st = np.zeros(max(B, 1), dtype=np.int32)
        worst = self._L.tgms_solve_batch_multi(self._h, B, _ptr(so), _ptr(W), _ptr(T), _ptr(ED), _ptr(C), _ptr(st))
        if worst in (_lib.ERR_DEVICE, _lib.ERR_NO_DEVICE):
            raise TgmsError(worst, self.last_error())
        return C, st[:B], worst

    def sample(self, seg_offsets, waypoints, seg_times, end_derivs, coeffs, dt: float,
               yaw_mode: int = _lib.YAW_CONSTANT, yaw_const: float = 0.0):
        so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
        W = np.ascontiguousarray(waypoints, dtype=np.float64).reshape(-1, 3)
        T = np.ascontiguousarray(seg_times, dtype=np.float64).reshape(-1)
        ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64).reshape(-1, 18)
        C = np.ascontiguousarray(coeffs, dtype=np.float64)
        B = so.shape[0] - 1
        offs = sample_offsets(so, T, dt)
        out = np.zeros((int(offs[-1]), _lib.GOAL_STRIDE), dtype=np.float64)
        st = self._L.tgms_sample_batch(self._h, B, _ptr(so), _ptr(W), _ptr(T), _ptr(ED), _ptr(C), float(dt),
                                       int(yaw_mode), float(yaw_const), _ptr(offs), _ptr(out))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())
        return offs, out

    def refine(self, seg_offsets, waypoints, seg_times, end_derivs=None, k_T: float = 1.0, eta: float = 0.1,
               iters: int = 10, coeffs: bool = True):
        """Time-allocation refinement on the GPU (include/tgms.h tgms_refine_batch).
        Returns (T [S], coeffs [S,3,8] or None, cost [B], status [B], worst)."""
        so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
        W = np.ascontiguousarray(waypoints, dtype=np.float64).reshape(-1, 3)
        T = np.array(seg_times, dtype=np.float64).reshape(-1)
        ED = None if end_derivs is None else np.ascontiguousarray(end_derivs, dtype=np.float64).reshape(-1, 18)
        B = so.shape[0] - 1
        C = np.zeros((int(so[-1]), 3, 8), dtype=np.float64) if coeffs else None
        cost = np.zeros(max(B, 1), dtype=np.float64)
        st = np.zeros(max(B, 1), dtype=np.int32)
        worst = self._L.tgms_refine_batch(self._h, B, _ptr(so), _ptr(W), _ptr(T), _ptr(ED), float(k_T), float(eta),
                                          int(iters), _ptr(C), _ptr(cost), _ptr(st))
        if worst in (_lib.ERR_DEVICE, _lib.ERR_NO_DEVICE):
            raise TgmsError(worst, self.last_error())
        return T, C, cost[:B], st[:B], worst

    # -------------------------------------------------------------- device API
    def refine_uniform_device(self, B: int, M: int, d_waypoints, d_seg_times, d_seg_times_out, k_T: float,
                              eta: float, d_cost=None, d_status=None, d_end_derivs=None, stream: int = 0) -> None:
        st = self._L.tgms_refine_uniform_device(self._h, int(B), int(M), _ptr(d_waypoints), _ptr(d_seg_times),
                                                _ptr(d_end_derivs), float(k_T), float(eta), _ptr(d_seg_times_out),
                                                _ptr(d_cost), _ptr(d_status), ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def refine_loop_device(self, h_seg_offsets, d_seg_offsets, d_waypoints, d_seg_times, k_T: float, eta: float,
                           iters: int, d_coeffs=None, d_cost=None, d_status=None, d_end_derivs=None,
                           stream: int = 0) -> None:
        so = np.ascontiguousarray(h_seg_offsets, dtype=np.int32)
        st = self._L.tgms_refine_loop_device(self._h, int(so.shape[0] - 1), _ptr(so), _ptr(d_seg_offsets),
                                             _ptr(d_waypoints), _ptr(d_seg_times), _ptr(d_end_derivs), float(k_T),
                                             float(eta), int(iters), _ptr(d_coeffs), _ptr(d_cost), _ptr(d_status),
                                             ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def refine_batch_device(self, h_seg_offsets, d_seg_offsets, d_waypoints, d_seg_times, d_seg_times_out,
                            k_T: float, eta: float, d_cost=None, d_status=None, d_end_derivs=None,
                            stream: int = 0) -> None:
        so = np.ascontiguousarray(h_seg_offsets, dtype=np.int32)
        st = self._L.tgms_refine_batch_device(self._h, int(so.shape[0] - 1), _ptr(so), _ptr(d_seg_offsets),
                                              _ptr(d_waypoints), _ptr(d_seg_times), _ptr(d_end_derivs), float(k_T),
                                              float(eta), _ptr(d_seg_times_out), _ptr(d_cost), _ptr(d_status),
                                              ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def solve_uniform_device(self, B: int, M: int, d_waypoints, d_seg_times, d_coeffs, d_status=None,
                             d_end_derivs=None, stream: int = 0) -> None:
        st = self._L.tgms_solve_uniform_device(self._h, int(B), int(M), _ptr(d_waypoints), _ptr(d_seg_times),
                                               _ptr(d_end_derivs), _ptr(d_coeffs), _ptr(d_status),
                                               ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def solve_batch_device(self, h_seg_offsets, d_seg_offsets, d_waypoints, d_seg_times, d_coeffs,
                           d_status=None, d_end_derivs=None, stream: int = 0) -> None:
        so = np.ascontiguousarray(h_seg_offsets, dtype=np.int32)
        st = self._L.tgms_solve_batch_device(self._h, int(so.shape[0] - 1), _ptr(so), _ptr(d_seg_offsets),
                                             _ptr(d_waypoints), _ptr(d_seg_times), _ptr(d_end_derivs),
                                             _ptr(d_coeffs), _ptr(d_status), ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def solve_batch_multi_device(self, h_seg_offsets, d_seg_offsets, d_waypoints, d_seg_times, d_coeffs,
                                 d_status=None, d_end_derivs=None, stream: int = 0) -> None:
        so = np.ascontiguousarray(h_seg_offsets, dtype=np.int32)
        st = self._L.tgms_solve_batch_multi_device(self._h, int(so.shape[0] - 1), _ptr(so), _ptr(d_seg_offsets),
                                                   _ptr(d_waypoints), _ptr(d_seg_times), _ptr(d_end_derivs),
                                                   _ptr(d_coeffs), _ptr(d_status), ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def refine_loop_multi_device(self, h_seg_offsets, d_seg_offsets, d_waypoints, d_seg_times, k_T: float,
                                 eta: float, iters: int, d_coeffs=None, d_cost=None, d_status=None,
                                 d_end_derivs=None, stream: int = 0) -> None:
        so = np.ascontiguousarray(h_seg_offsets, dtype=np.int32)
        st = self._L.tgms_refine_loop_multi_device(self._h, int(so.shape[0] - 1), _ptr(so), _ptr(d_seg_offsets),
                                                   _ptr(d_waypoints), _ptr(d_seg_times), _ptr(d_end_derivs),
                                                   float(k_T), float(eta), int(iters), _ptr(d_coeffs),
                                                   _ptr(d_cost), _ptr(d_status), ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())

    def sample_device(self, B: int, d_seg_offsets, d_waypoints, d_seg_times, d_coeffs, dt: float,
                      d_sample_offsets, d_out, d_end_derivs=None, yaw_mode: int = _lib.YAW_CONSTANT,
                      yaw_const: float = 0.0, stream: int = 0) -> None:
        st = self._L.tgms_sample_batch_device(self._h, int(B), _ptr(d_seg_offsets), _ptr(d_waypoints),
                                              _ptr(d_seg_times), _ptr(d_end_derivs), _ptr(d_coeffs), float(dt),
                                              int(yaw_mode), float(yaw_const), _ptr(d_sample_offsets),
                                              _ptr(d_out), ctypes.c_void_p(stream))
        if st != _lib.OK:
            raise TgmsError(st, self.last_error())


def sample_count(total_T: float, dt: float) -> int:
    return int(_lib.load().tgms_sample_count(float(total_T), float(dt)))


def sample_offsets(seg_offsets, seg_times, dt: float) -> np.ndarray:
    so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
    T = np.ascontiguousarray(seg_times, dtype=np.float64).reshape(-1)
    B = so.shape[0] - 1
    offs = np.zeros(B + 1, dtype=np.int64)
    st = _lib.load().tgms_sample_offsets(B, _ptr(so), _ptr(T), float(dt), _ptr(offs))
    if st != _lib.OK:
        raise TgmsError(st, "tgms_sample_offsets")
    return offs


def plan_shards(seg_offsets, parts: int, method: int = _lib.METHOD_REDUCED) -> np.ndarray:
    """tgms_plan_shards (host only): [parts+1] contiguous cost-balanced trajectory bounds."""
    so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
    bounds = np.zeros(int(parts) + 1, dtype=np.int32)
    st = _lib.load().tgms_plan_shards(int(so.shape[0] - 1), _ptr(so), int(parts), int(method), _ptr(bounds))
    if st != _lib.OK:
        raise TgmsError(st, "tgms_plan_shards")
    return bounds


def multi_schedule(seg_offsets, device_count: int, method: int = _lib.METHOD_REDUCED, flags: int = 0):
    """tgms_multi_schedule (host only): the multi-GPU call's whole schedule -- shard bounds,
    per-device workspace sizes, pieces and transfers (lists of dicts, issue order)."""
    import ctypes
    L = _lib.load()
    so = np.ascontiguousarray(seg_offsets, dtype=np.int32)
    B = int(so.shape[0] - 1)
    n = int(device_count)
    bounds = np.zeros(n + 1, dtype=np.int32)
    ws = np.zeros(n, dtype=np.int64)
    npc, nx = ctypes.c_int32(0), ctypes.c_int32(0)
    st = L.tgms_multi_schedule(n, B, _ptr(so), int(method), int(flags), _ptr(bounds), _ptr(ws), None, 0,
                               ctypes.byref(npc), None, 0, ctypes.byref(nx))
    if st not in (_lib.OK, _lib.ERR_INVALID_ARG) or (st != _lib.OK and npc.value == 0 and nx.value == 0):
        raise TgmsError(st, "tgms_multi_schedule")
    pieces = (_lib.Piece * max(1, npc.value))()
    xfers = (_lib.Xfer * max(1, nx.value))()
    st = L.tgms_multi_schedule(n, B, _ptr(so), int(method), int(flags), _ptr(bounds), _ptr(ws), pieces, npc.value,
                               ctypes.byref(npc), xfers, nx.value, ctypes.byref(nx))
    if st != _lib.OK:
        raise TgmsError(st, "tgms_multi_schedule")
    P = [{"dev": p.dev, "piece": p.piece, "lo": p.lo, "hi": p.hi, "s0": p.s0, "s1": p.s1,
          "ws_off": list(p.ws_off)} for p in pieces[: npc.value]]
    X = [{f: getattr(x, f) for f, _ in _lib.Xfer._fields_} for x in xfers[: nx.value]]
    return bounds, ws, P, X
