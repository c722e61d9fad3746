#!/usr/bin/env python3
"""Config 5 at full size (1,048,576 ragged) through tgms_refine_loop_multi_device on one
device: every call timed alone (synchronised before and after: HIP events on the launch
stream, host time of the call), then K calls back to back (pipelined wall time)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

so, W, T = S.ragged_batch(1048576, 2, 16)
B, Sg = len(so) - 1, int(so[-1])
d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda(0)
dso, dW, T0 = d(so), d(W), d(T)
dT = torch.empty_like(T0)
dC = torch.empty((Sg, 3, 8), dtype=torch.float64, device="cuda:0")
dcost = torch.empty((B,), dtype=torch.float64, device="cuda:0")
dst = torch.full((B,), -1, dtype=torch.int32, device="cuda:0")
st = torch.cuda.current_stream(0)
mh = Solver(device_count=int(os.environ.get("C5F_DEV", "1")))
rows = []
for i in range(6):
    dT.copy_(T0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    h0 = time.perf_counter()
    mh.refine_loop_multi_device(so, dso, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=st.cuda_stream)
    hh = (time.perf_counter() - h0) * 1e3
    e1.record(st)
    torch.cuda.synchronize()
    rows.append({"call": i, "ms_events": e0.elapsed_time(e1), "host_ms": hh})
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    dT.copy_(T0)
    mh.refine_loop_multi_device(so, dso, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=st.cuda_stream)
torch.cuda.synchronize()
print(json.dumps({"calls": rows, "pipelined_ms": (time.perf_counter() - t0) / 5 * 1e3,
                  "bad": int((dst != 0).sum().item())}))
