#!/usr/bin/env python3
"""Sampler micro-benchmark: config-3 trajectories (first N) at dt, both yaw modes."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import YAW_CONSTANT, YAW_VELOCITY
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver, sample_offsets

N = int(os.environ.get("SB_N", 4096)); M = 10; dt = float(os.environ.get("SB_DT", 0.01))
_, W, T = S.uniform_batch(N, M)
if os.environ.get("SB_CONST_T"):  # equal-length trajectories: no tail imbalance
    T[:] = float(os.environ["SB_CONST_T"])
s = Solver(0)
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((N, M, 3, 8), dtype=torch.float64, device="cuda")
s.solve_uniform_device(N, M, dW, dT, dC)
so = np.arange(N + 1, dtype=np.int32) * M
offs = sample_offsets(so, T.reshape(-1), dt)
d_so, d_offs = torch.from_numpy(so).cuda(), torch.from_numpy(offs).cuda()
out = torch.empty((int(offs[-1]), 14), dtype=torch.float64, device="cuda")
for mode, name in ((YAW_CONSTANT, "constant"), (YAW_VELOCITY, "velocity")):
    run = lambda: s.sample_device(N, d_so, dW, dT, dC, dt, d_offs, out, yaw_mode=mode)
    run(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): run()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"yaw": name, "samples": int(offs[-1]), "ms": ms, "GBs": int(offs[-1]) * 112 / ms / 1e6}))
