#!/usr/bin/env python3
"""Phase timeline of the reduced kernel from a TGMS_STAMPS build (TGMS_LIB):
per-wave s_memtime at start / staged / chain done / interface done / backsub done /
end, plus XCC id and HW_ID (s_memtime is per XCD, so spans are taken per XCD)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd.solver import Solver
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd import _lib

B = int(os.environ.get("KB_B", 65536)); M = int(os.environ.get("KB_M", 10))
so, W, T = S.uniform_batch(B, M)
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
s = Solver(0)
for _ in range(20):
    s.solve_uniform_device(B, M, dW, dT, dC, dS)
torch.cuda.synchronize()
L = _lib.load()
TPW = int(os.environ.get("KB_TPW", 64))  # trajectories per wave of the stamped kernel
nw = (B + TPW - 1) // TPW
buf = (ctypes.c_ulonglong * (nw * 16))()
L.tgms_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.tgms_debug_stamps(buf, nw * 16)
st = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 16).astype(np.int64)
st = st[(st[:, 0] != 0) & (st[:, 5] != 0)]
nw = st.shape[0]
rt = st[:, 6:8]
clk = (st[:, 5] - st[:, 0]).sum() / max(((rt[:, 1] - rt[:, 0]) * 10).sum(), 1)  # cycles per ns
xcc = st[:, 8] & 0xF
hw = st[:, 9]
ph = np.diff(st[:, :6], axis=1)
names = (["stage_T", "factor", "stage_W", "forward", "back+emit"] if TPW == 64 else
         ["load+stage", "chain", "interface", "backsub", "emission"])
out = {"waves": int(nw), "clock_GHz": float(clk),
       "phase_us_mean": {n: float(ph[:, i].mean() / clk / 1e3) for i, n in enumerate(names)},
       "wave_life_us_mean": float((st[:, 5] - st[:, 0]).mean() / clk / 1e3)}
per = []
for x in range(8):
    m = xcc == x
    if not m.any():
        continue
    t0 = st[m, 0].min()
    starts = (st[m, 0] - t0) / clk / 1e3
    ends = (st[m, 5] - t0) / clk / 1e3
    per.append({"xcc": x, "waves": int(m.sum()), "span_us": float(ends.max()),
                "start_q": [round(float(np.percentile(starts, q)), 2) for q in (0, 10, 50, 90, 100)],
                "end_q": [round(float(np.percentile(ends, q)), 2) for q in (0, 10, 50, 90, 100)]})
out["per_xcd"] = per
# realtime (global 100 MHz) spans
r0 = rt[:, 0].min()
out["realtime_span_us"] = float((rt[:, 1].max() - r0) / 100.0)
out["realtime_start_q_us"] = [round(float(np.percentile((rt[:, 0] - r0) / 100.0, q)), 2) for q in (0, 10, 50, 90, 100)]
out["realtime_end_q_us"] = [round(float(np.percentile((rt[:, 1] - r0) / 100.0, q)), 2) for q in (0, 10, 50, 90, 100)]
print(json.dumps(out, indent=None))
