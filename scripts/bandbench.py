#!/usr/bin/env python3
"""Band-KKT kernel timing for one libtgms build (TGMS_LIB selects it): config 3
(65,536 x M = 10, KB_B / KB_M override), median of 10 launches, max rel. difference
to the reduced solve of the same build."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_REDUCED, synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B = int(os.environ.get("KB_B", 65536)); M = int(os.environ.get("KB_M", 10)); K = 10
_, W, T = S.uniform_batch(B, M)
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda"); dR = torch.empty_like(dC)
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
s = Solver(0)
s.solve_uniform_device(B, M, dW, dT, dR, dS)
s.set_method(METHOD_BAND_KKT)
s.solve_uniform_device(B, M, dW, dT, dC, dS)
torch.cuda.synchronize()
ts = []
for _ in range(K):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); s.solve_uniform_device(B, M, dW, dT, dC, dS); e1.record()
    torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
err = ((dC - dR).abs().amax(dim=(1, 3)) / dR.abs().amax(dim=(1, 3))).max().item()
print(json.dumps({"lib": os.path.basename(os.environ.get("TGMS_LIB", "default")), "B": B, "M": M,
                  "median_ms": sorted(ts)[K // 2], "traj_per_s": B / (sorted(ts)[K // 2] * 1e-3),
                  "max_rel_diff_vs_reduced": err, "status_ok": bool((dS == 0).all().item())}))
