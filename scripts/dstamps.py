#!/usr/bin/env python3
"""Per-step phase profile of the dense-KKT kernel from a TGMS_DENSE_STAMPS build
(TGMS_LIB): wave 0 of blocks < 64 stamps s_memtime at step start / pivot chosen /
multipliers + right-hand side done / own rows updated; the barrier wait is the gap to
the next step.  Prints mean cycles per phase, summed over the steps."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd.solver import Solver
METHOD_DENSE_KKT = __import__("trajectory_generator_ros2_amd._lib", fromlist=["x"]).METHOD_DENSE_KKT
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd import _lib

B = int(os.environ.get("KB_B", 65536)); M = int(os.environ.get("KB_M", 10))
N = 14 * M + 2
so, W, T = S.uniform_batch(B, M)
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
s = Solver(0, METHOD_DENSE_KKT)
s.solve_uniform_device(B, M, dW, dT, dC, dS)
torch.cuda.synchronize()
L = _lib.load()
NB, NS = 64, 160
buf = (ctypes.c_ulonglong * (NB * NS * 4))()
L.tgms_debug_dense_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.tgms_debug_dense_stamps(buf, NB * NS * 4)
st = np.frombuffer(buf, dtype=np.uint64).reshape(NB, NS, 4).astype(np.int64)
steps = st[:, :N, :]
nxt = np.concatenate([st[:, 1:N, 0], st[:, N:N + 1, 0]], axis=1)  # next step start (or LU end)
ph = {"pivot": steps[:, :, 1] - steps[:, :, 0], "u+rhs": steps[:, :, 2] - steps[:, :, 1],
      "update": steps[:, :, 3] - steps[:, :, 2], "barrier": nxt - steps[:, :, 3]}
out = {k: float(v.sum(axis=1).mean()) for k, v in ph.items()}
out["assembly"] = float((st[:, 0, 0] - st[:, N + 1, 0]).mean())
out["backsub"] = float((st[:, N, 1] - st[:, N, 0]).mean())
out["total"] = float((st[:, N, 1] - st[:, N + 1, 0]).mean())
q = [0, 10, 40, 80, 120, N - 1]
out["per_step_update"] = {int(k): float(ph["update"][:, k].mean()) for k in q}
out["per_step_pivot"] = {int(k): float(ph["pivot"][:, k].mean()) for k in q}
print(json.dumps(out, indent=1))
