#!/usr/bin/env python3
"""Refinement-loop timing (10 steps + cost + final solve) through tgms_refine_loop_device
for a uniform (65,536 x M = 10) and a ragged (M ~ U{2..16}) batch; set
TGMS_REFINE_STEPWISE=1 for the one-launch-per-step path."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

s = Solver(0)
res = {"stepwise": bool(os.environ.get("TGMS_REFINE_STEPWISE")), "lib": os.path.basename(os.environ.get("TGMS_LIB", "default"))}
NB = int(os.environ.get("REF_B", "65536"))
for name, (so, W, T) in {"uniform_M10": S.uniform_batch(NB, 10), "ragged_2_16": S.ragged_batch(NB, 2, 16)}.items():
    so = np.asarray(so, dtype=np.int32)
    d_so = torch.from_numpy(so).cuda()
    dW = torch.from_numpy(np.ascontiguousarray(W).reshape(-1, 3)).cuda()
    T0 = torch.from_numpy(np.ascontiguousarray(T).reshape(-1)).cuda()
    dT = torch.empty_like(T0)
    dC = torch.empty((int(so[-1]), 3, 8), dtype=torch.float64, device="cuda")
    dcost = torch.empty(len(so) - 1, dtype=torch.float64, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream

    def run():
        dT.copy_(T0)
        s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, stream=sp)

    run(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    res[name + "_ms"] = (time.perf_counter() - t0) / 5 * 1e3
print(json.dumps(res))
