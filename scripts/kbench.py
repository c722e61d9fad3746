#!/usr/bin/env python3
"""Kernel micro-benchmark for one libtgms build (TGMS_LIB selects it):
time the reduced solve at config 3 and check it against the oracle (reduced fp64)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd.solver import Solver
from trajectory_generator_ros2_amd import synthetic as S

B = int(os.environ.get("KB_B", 65536)); M = int(os.environ.get("KB_M", 10)); K = int(os.environ.get("KB_K", 30))
METHOD = int(os.environ.get("KB_METHOD", 0))  # 0 reduced, 1 dense KKT, 2 band KKT
so, W, T = S.uniform_batch(B, M)
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
s = Solver(0)
s.set_method(METHOD)
sp = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    s.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
torch.cuda.synchronize()
e0 = [torch.cuda.Event(enable_timing=True) for _ in range(K)]; e1 = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
ROT = int(os.environ.get("KB_ROT", 1))  # >1: a fresh batch every launch (beyond the Infinity Cache)
sets = [(dW, dT, dC)]
for i in range(1, ROT):
    _, Wi, Ti = S.uniform_batch(B, M, seed=S.SEED + 1000 + i)
    sets.append((torch.from_numpy(Wi).cuda(), torch.from_numpy(Ti).cuda(), torch.empty_like(dC)))
for k in range(ROT):
    s.solve_uniform_device(B, M, *sets[k][:2], sets[k][2], dS, stream=sp)
for k in range(K):
    a, b_, c_ = sets[k % ROT]
    e0[k].record(); s.solve_uniform_device(B, M, a, b_, c_, dS, stream=sp); e1[k].record()
torch.cuda.synchronize()
s.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
torch.cuda.synchronize()
ms = sorted(e0[k].elapsed_time(e1[k]) for k in range(K))
C = dC.cpu().numpy()
ref_path = f"/tmp/ref_{B}_{M}.npy"
if os.path.exists(ref_path):
    R = np.load(ref_path)
else:
    from oracle import oracle as O
    R, _ = O.solve_batch(so, W.reshape(-1, 3), T.reshape(-1), None, O.KKT_C4, 16)
    R = R.reshape(B, M, 3, 8); np.save(ref_path, R)
errs = np.abs(C - R).max(axis=(1, 3)) / np.abs(R).max(axis=(1, 3))
err = float(errs.max())
bad = np.argwhere(errs > 1e-9)
if len(bad):
    print(json.dumps({"n_bad": int(len(bad)), "first_bad": bad[:8].tolist(),
                      "worst": np.unravel_index(int(errs.argmax()), errs.shape)[0].item()}), file=sys.stderr)
print(json.dumps({"lib": os.path.basename(os.environ.get("TGMS_LIB", "default")), "B": B, "M": M, "rot": ROT,
                  "method": METHOD,
                  "median_us": ms[K // 2] * 1e3, "min_us": ms[0] * 1e3,
                  "traj_per_s": B / (ms[K // 2] * 1e-3), "max_rel_err": err,
                  "status_ok": bool((dS == 0).all().item())}))
