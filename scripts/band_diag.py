#!/usr/bin/env python3
"""Band-KKT diagnosis: which trajectories of a uniform batch disagree with the reduced solve
(KB_B x KB_M), grouped by 16-trajectory group and slot."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import METHOD_BAND_KKT, synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B = int(os.environ.get("KB_B", 20001)); M = int(os.environ.get("KB_M", 3))
_, W, T = S.uniform_batch(B, M, seed=int(os.environ.get("KB_SEED", 910)))
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda"); dR = torch.empty_like(dC)
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
s = Solver(0)
s.solve_uniform_device(B, M, dW, dT, dR, dS)
s.set_method(METHOD_BAND_KKT)
s.solve_uniform_device(B, M, dW, dT, dC, dS)
torch.cuda.synchronize()
err = ((dC - dR).abs().amax(dim=(1, 3)) / dR.abs().amax(dim=(1, 3))).amax(dim=1).cpu().numpy()
bad = np.nonzero(err > 1e-9)[0]
out = {"B": B, "M": M, "n_bad": int(bad.size), "first": bad[:20].tolist(),
       "slots": np.bincount(bad % 16, minlength=16).tolist(),
       "groups_min_max": [int(bad.min() // 16), int(bad.max() // 16)] if bad.size else None,
       "iters": np.bincount(bad // 16 // 2048).tolist() if bad.size else [],
       "wave_hist_mod8": np.bincount((bad // 16 % 2048) % 8, minlength=8).tolist() if bad.size else [],
       "waves_distinct": int(np.unique(bad // 16 % 2048).size) if bad.size else 0,
       "max_err": float(err.max()),
       "status_nonzero": int((dS != 0).sum().item())}
print(json.dumps(out))
