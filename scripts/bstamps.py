#!/usr/bin/env python3
"""Per-step phase profile of the band-KKT forward elimination from a TGMS_BAND_STAMPS
build (TGMS_LIB): lane 0 of blocks < 64, first trajectory pair, s_memtime (after
draining its memory counters) at: step start / pivot searched / rows interchanged /
multipliers published / update done / U row stored / entering row assembled."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import METHOD_BAND_KKT, _lib, synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B, M = 65536, 10
N = 14 * M + 2
_, W, T = S.uniform_batch(B, M)
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
s = Solver(0, METHOD_BAND_KKT)
for _ in range(2):
    s.solve_uniform_device(B, M, dW, dT, dC, None)
torch.cuda.synchronize()
L = _lib.load()
NB, NS, NP = 64, 160, 8
buf = (ctypes.c_ulonglong * (NB * NS * NP))()
L.tgms_debug_band_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.tgms_debug_band_stamps(buf, NB * NS * NP)
st = np.frombuffer(buf, dtype=np.uint64).reshape(NB, NS, NP).astype(np.int64)[:, :N - 1]
names = ["pivot_search", "interchange", "multipliers", "slot_read+update", "U_store", "entering_row"]
out = {n: float(np.median((st[:, :, i + 1] - st[:, :, i]).mean(axis=1))) for i, n in enumerate(names)}
out["to_next_step"] = float(np.median((st[:, 1:, 0] - st[:, :-1, 6]).mean(axis=1)))
out["step_total"] = float(np.median((st[:, 1:, 0] - st[:, :-1, 0]).mean(axis=1)))
print(json.dumps({"cycles_per_step_mean_over_steps_median_over_blocks": out}))
