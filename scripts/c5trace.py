#!/usr/bin/env python3
"""Config-5 timing breakdown: host time per tgms_refine_loop_device call vs GPU time
(events), for iters = 0 (final solve only) and 10; run under rocprofv3 --kernel-trace
to see the per-group kernel timeline."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B = int(os.environ.get("C5_B", 65536))
so, W, T = S.ragged_batch(B, 2, 16)
dev = 0
d_so = torch.from_numpy(so.astype(np.int32)).to(dev)
dW = torch.from_numpy(W.reshape(-1, 3)).to(dev)
T0 = torch.from_numpy(T.reshape(-1)).to(dev)
dT = torch.empty_like(T0)
dC = torch.empty((int(so[-1]), 3, 8), dtype=torch.float64, device=dev)
dcost = torch.empty(B, dtype=torch.float64, device=dev)
s = Solver(dev)
sp = torch.cuda.current_stream().cuda_stream
out = {}
for iters in (0, 1, 10):
    for _ in range(2):
        dT.copy_(T0); s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, iters, dC, dcost, stream=sp)
    torch.cuda.synchronize()
    hs, gs = [], []
    for _ in range(5):
        dT.copy_(T0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter(); e0.record()
        s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, iters, dC, dcost, stream=sp)
        t1 = time.perf_counter(); e1.record()
        torch.cuda.synchronize()
        hs.append((t1 - t0) * 1e3); gs.append(e0.elapsed_time(e1))
    out[iters] = {"host_submit_ms": float(np.median(hs)), "gpu_ms": float(np.median(gs))}
print(json.dumps(out))
