#!/usr/bin/env python3
"""Config-5 loop through tgms_refine_loop_device, results saved to argv[1] (.npz):
run once with and once without TGMS_REFINE_STEPWISE and compare the files."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

out = {}
rng = np.random.default_rng(3)
for name, (B, ed) in {"plain": (65536, False), "ed": (5000, True)}.items():
    so, W, T = S.ragged_batch(B, 1, 16, seed=11)
    T = T.reshape(-1).copy()
    T[so[7]] = -1.0  # one invalid trajectory
    d_so = torch.from_numpy(so.astype(np.int32)).cuda()
    dW = torch.from_numpy(W.reshape(-1, 3)).cuda()
    dT = torch.from_numpy(T).cuda()
    dC = torch.empty((int(so[-1]), 3, 8), dtype=torch.float64, device="cuda")
    dcost = torch.empty(B, dtype=torch.float64, device="cuda")
    dst = torch.empty(B, dtype=torch.int32, device="cuda")
    dED = torch.from_numpy(rng.normal(size=(B, 18))).cuda() if ed else None
    s = Solver(0)
    s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, d_end_derivs=dED)
    torch.cuda.synchronize()
    out[name + "_T"] = dT.cpu().numpy(); out[name + "_C"] = dC.cpu().numpy()
    out[name + "_cost"] = dcost.cpu().numpy(); out[name + "_st"] = dst.cpu().numpy()
    s.close()
np.savez(sys.argv[1], **out)
