"""ctypes binding of libtgms.so (the C ABI declared in include/tgms.h).

This is the Python-side twin of the binding a ROS maintainer would add (see
INTEGRATION.md).  It loads ONLY the in-tree HIP library; if that library is
missing or cannot be loaded the import fails loudly — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

from .build import LIB_TGMS

OK, ERR_INVALID_ARG, ERR_SINGULAR, ERR_NONFINITE, ERR_NO_DEVICE, ERR_DEVICE, ERR_UNSUPPORTED, ERR_SKIPPED = range(8)
METHOD_REDUCED, METHOD_DENSE_KKT, METHOD_BAND_KKT = 0, 1, 2
YAW_CONSTANT, YAW_VELOCITY = 0, 1
ABI_VERSION = 2
MAX_SEGMENTS = 16
DENSE_MAX_SEGMENTS = 10
GOAL_STRIDE = 14

# Every symbol include/tgms.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = [
    "tgms_abi_version", "tgms_status_string", "tgms_create", "tgms_create_host", "tgms_destroy", "tgms_last_error",
    "tgms_set_method", "tgms_solve_batch", "tgms_solve_uniform_device", "tgms_solve_batch_device",
    "tgms_sample_count", "tgms_sample_offsets", "tgms_sample_batch", "tgms_sample_batch_device",
    "tgms_refine_uniform_device", "tgms_refine_batch_device", "tgms_refine_loop_device", "tgms_refine_batch",
    "tgms_create_multi", "tgms_device_count", "tgms_plan_shards", "tgms_solve_batch_multi",
    "tgms_solve_batch_multi_device", "tgms_refine_loop_multi_device", "tgms_multi_schedule",
]

SCHED_REFINE, SCHED_END_DERIVS, SCHED_COEFFS, SCHED_STATUS, SCHED_COST, SCHED_SELF_GATHER = 1, 2, 4, 8, 16, 32


class Piece(ctypes.Structure):
    """tgms_piece (include/tgms.h): one piece of one device's shard."""
    _fields_ = [("dev", ctypes.c_int32), ("piece", ctypes.c_int32), ("lo", ctypes.c_int32), ("hi", ctypes.c_int32),
                ("s0", ctypes.c_int64), ("s1", ctypes.c_int64), ("ws_off", ctypes.c_int64 * 11)]


class Xfer(ctypes.Structure):
    """tgms_xfer (include/tgms.h): one ncclSend/ncclRecv pair of the multi-GPU schedule."""
    _fields_ = [("dev", ctypes.c_int32), ("piece", ctypes.c_int32), ("gather", ctypes.c_int32),
                ("array", ctypes.c_int32), ("batch_elem", ctypes.c_int64), ("ws_byte", ctypes.c_int64),
                ("count", ctypes.c_int64), ("elem_bytes", ctypes.c_int32), ("group", ctypes.c_int32)]

_lib = None


class TgmsError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        self.status = status
        super().__init__(f"{status_string(status)}: {msg}" if msg else status_string(status))


def load(path: str = ""):
    """Load libtgms.so.  Raises if it is absent: build it with __graft_entry__.build().
    TGMS_LIB may name an alternative build of the same ABI (kernel experiments)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("TGMS_LIB", "") or LIB_TGMS
    if not os.path.exists(path):
        raise ImportError(f"libtgms.so not built at {path}; run `python -c 'import __graft_entry__ as g; g.build()'`")
    # PyTorch-ROCm ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Load
    # torch first so libtgms binds to the HIP runtime instance torch uses: one runtime
    # per process, so device pointers and streams are shared between the two.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    L.tgms_abi_version.restype = ctypes.c_int
    L.tgms_status_string.argtypes = [ctypes.c_int]
    L.tgms_status_string.restype = ctypes.c_char_p
    L.tgms_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.tgms_create.restype = ctypes.c_int
    L.tgms_create_host.argtypes = [ctypes.POINTER(vp)]
    L.tgms_create_host.restype = ctypes.c_int
    L.tgms_destroy.argtypes = [vp]
    L.tgms_destroy.restype = None
    L.tgms_last_error.argtypes = [vp]
    L.tgms_last_error.restype = ctypes.c_char_p
    L.tgms_set_method.argtypes = [vp, ctypes.c_int]
    L.tgms_set_method.restype = ctypes.c_int
    L.tgms_solve_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
    L.tgms_solve_batch.restype = ctypes.c_int
    L.tgms_solve_uniform_device.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, vp]
    L.tgms_solve_uniform_device.restype = ctypes.c_int
    L.tgms_solve_batch_device.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tgms_solve_batch_device.restype = ctypes.c_int
    L.tgms_sample_count.argtypes = [dbl, dbl]
    L.tgms_sample_count.restype = i64
    L.tgms_sample_offsets.argtypes = [i32, vp, vp, dbl, vp]
    L.tgms_sample_offsets.restype = ctypes.c_int
    L.tgms_sample_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, ctypes.c_int, dbl, vp, vp]
    L.tgms_sample_batch.restype = ctypes.c_int
    L.tgms_sample_batch_device.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, ctypes.c_int, dbl, vp, vp, vp]
    L.tgms_sample_batch_device.restype = ctypes.c_int
    L.tgms_refine_uniform_device.argtypes = [vp, i32, i32, vp, vp, vp, dbl, dbl, vp, vp, vp, vp]
    L.tgms_refine_uniform_device.restype = ctypes.c_int
    L.tgms_refine_batch_device.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, dbl, vp, vp, vp, vp]
    L.tgms_refine_batch_device.restype = ctypes.c_int
    L.tgms_refine_loop_device.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, dbl, i32, vp, vp, vp, vp]
    L.tgms_refine_loop_device.restype = ctypes.c_int
    L.tgms_refine_batch.argtypes = [vp, i32, vp, vp, vp, vp, dbl, dbl, i32, vp, vp, vp]
    L.tgms_refine_batch.restype = ctypes.c_int
    L.tgms_create_multi.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.tgms_create_multi.restype = ctypes.c_int
    L.tgms_device_count.argtypes = [vp]
    L.tgms_device_count.restype = ctypes.c_int
    L.tgms_plan_shards.argtypes = [i32, vp, i32, ctypes.c_int, vp]
    L.tgms_plan_shards.restype = ctypes.c_int
    L.tgms_solve_batch_multi.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
    L.tgms_solve_batch_multi.restype = ctypes.c_int
    L.tgms_solve_batch_multi_device.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp]
    L.tgms_solve_batch_multi_device.restype = ctypes.c_int
    L.tgms_refine_loop_multi_device.argtypes = [vp, i32, vp, vp, vp, vp, vp, dbl, dbl, i32, vp, vp, vp, vp]
    L.tgms_refine_loop_multi_device.restype = ctypes.c_int
    L.tgms_multi_schedule.argtypes = [i32, i32, vp, ctypes.c_int, i32, vp, vp, vp, i32, vp, vp, i32, vp]
    L.tgms_multi_schedule.restype = ctypes.c_int
    if L.tgms_abi_version() != ABI_VERSION:
        raise ImportError(f"libtgms ABI {L.tgms_abi_version()} != {ABI_VERSION}")
    _lib = L
    return L


def status_string(status: int) -> str:
    return load().tgms_status_string(int(status)).decode()
