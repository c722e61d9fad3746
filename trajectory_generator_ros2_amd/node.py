"""ctypes binding of libtgms_node.so (include/tgms_node.h): the C++ MinSnap trajectory
behind the reference's Trajectory interface, driven the way TrajectoryGenerator drives
a primitive (readParameters -> generateTraj -> ... -> generateStopTraj on END).

Mirrors src/TrajectoryGenerator.cpp:150-425 (readParameters), :71 (generateTraj),
:516 (generateStopTraj) and :556-573 (pubCB reads goals[pub_index] and index_msgs).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .build import LIB_HOST, build_host

GOAL_FIELDS = 15  # p[3] v[3] a[3] j[3] psi dpsi power

NODE_EXPORTS = [
    "tgms_node_new", "tgms_node_free", "tgms_node_set_double", "tgms_node_set_array", "tgms_node_set_string",
    "tgms_node_read_parameters", "tgms_node_generate_traj", "tgms_node_generate_stop_traj",
    "tgms_node_pub_index", "tgms_node_goal_count", "tgms_node_goals", "tgms_node_frame_id",
    "tgms_node_index_keys", "tgms_node_index_msg", "tgms_node_inside_bounds", "tgms_node_coefficients",
    "tgms_node_dt", "tgms_node_shape_waypoints",
]

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_HOST):
        build_host()
    if not os.path.exists(LIB_HOST):
        raise ImportError(f"libtgms_node.so not built at {LIB_HOST}")
    from . import _lib as core
    core.load()  # libtgms (and torch's HIP runtime) first
    L = ctypes.CDLL(LIB_HOST)
    vp, i32, i64, dbl, cp = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_char_p
    sig = {
        "tgms_node_new": ([], vp), "tgms_node_free": ([vp], None),
        "tgms_node_set_double": ([vp, cp, dbl], None), "tgms_node_set_array": ([vp, cp, vp, i32], None),
        "tgms_node_set_string": ([vp, cp, cp], None), "tgms_node_read_parameters": ([vp], ctypes.c_int),
        "tgms_node_generate_traj": ([vp], i64), "tgms_node_generate_stop_traj": ([vp, i32], i64),
        "tgms_node_pub_index": ([vp], i32), "tgms_node_goal_count": ([vp], i64),
        "tgms_node_goals": ([vp, i64, i64, vp], ctypes.c_int), "tgms_node_frame_id": ([vp, i64], cp),
        "tgms_node_index_keys": ([vp, vp, i32], i32), "tgms_node_index_msg": ([vp, i32], cp),
        "tgms_node_inside_bounds": ([vp, dbl, dbl, dbl, dbl, dbl, dbl], ctypes.c_int),
        "tgms_node_coefficients": ([vp, vp, i32], i32), "tgms_node_dt": ([vp], dbl),
        "tgms_node_shape_waypoints": ([cp, dbl, dbl, dbl, dbl, dbl, dbl, i32, vp, i32], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def shape_waypoints(shape: str, cx=0.0, cy=0.0, orientation=0.0, length=1.0, width=1.0, z=0.0, laps=1):
    """[n, 3] waypoints of a reference polyline shape (host/factory.hpp shapeWaypoints)."""
    L = load()
    out = np.zeros((17, 3), dtype=np.float64)
    n = int(L.tgms_node_shape_waypoints(shape.encode(), cx, cy, orientation, length, width, z, int(laps),
                                        out.ctypes.data, 17))
    return out[:n]


class MinSnapNode:
    """Parameters in, goals out — the node-side view of a MinSnap trajectory."""

    def __init__(self, params: dict | None = None):
        self._L = load()
        self._n = self._L.tgms_node_new()
        for k, v in (params or {}).items():
            self.set(k, v)

    def close(self):
        if self._n:
            self._L.tgms_node_free(self._n)
            self._n = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set(self, name: str, value):
        key = name.encode()
        if isinstance(value, str):
            self._L.tgms_node_set_string(self._n, key, value.encode())
        elif np.ndim(value) == 0:
            self._L.tgms_node_set_double(self._n, key, float(value))
        else:
            a = np.ascontiguousarray(value, dtype=np.float64).reshape(-1)
            self._L.tgms_node_set_array(self._n, key, a.ctypes.data, int(a.size))

    def read_parameters(self) -> bool:
        return bool(self._L.tgms_node_read_parameters(self._n))

    @property
    def dt(self) -> float:
        return float(self._L.tgms_node_dt(self._n))

    def generate_traj(self) -> int:
        return int(self._L.tgms_node_generate_traj(self._n))

    def generate_stop_traj(self, pub_index: int) -> int:
        return int(self._L.tgms_node_generate_stop_traj(self._n, int(pub_index)))

    @property
    def pub_index(self) -> int:
        return int(self._L.tgms_node_pub_index(self._n))

    def goals(self) -> np.ndarray:
        n = int(self._L.tgms_node_goal_count(self._n))
        out = np.zeros((n, GOAL_FIELDS), dtype=np.float64)
        if n:
            assert self._L.tgms_node_goals(self._n, 0, n, out.ctypes.data)
        return out

    def frame_id(self, i: int) -> str:
        r = self._L.tgms_node_frame_id(self._n, int(i))
        return None if r is None else r.decode()

    def index_msgs(self) -> dict:
        cnt = int(self._L.tgms_node_index_keys(self._n, None, 0))
        keys = np.zeros(max(cnt, 1), dtype=np.int32)
        self._L.tgms_node_index_keys(self._n, keys.ctypes.data, cnt)
        return {int(k): self._L.tgms_node_index_msg(self._n, int(k)).decode() for k in keys[:cnt]}

    def inside_bounds(self, xmin, xmax, ymin, ymax, zmin, zmax) -> bool:
        return bool(self._L.tgms_node_inside_bounds(self._n, xmin, xmax, ymin, ymax, zmin, zmax))

    def coefficients(self) -> np.ndarray:
        cap = 16 * 24
        out = np.zeros(cap, dtype=np.float64)
        M = int(self._L.tgms_node_coefficients(self._n, out.ctypes.data, cap))
        return out[: M * 24].reshape(M, 3, 8)
