#!/usr/bin/env python3
"""Dense-KKT kernel A/B: time one libtgms build (TGMS_LIB) at KB_B x M for M in KB_MS and
save its coefficients (gpurun_out/dense_<tag>_M<M>.npy); with KB_CMP=tagA,tagB compare two
saved runs bit for bit instead."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

OUT = "gpurun_out"
if os.environ.get("KB_CMP"):
    a, b = os.environ["KB_CMP"].split(",")
    for f in sorted(os.listdir(OUT)):
        if f.startswith(f"dense_{a}_M"):
            A = np.load(os.path.join(OUT, f)); Bv = np.load(os.path.join(OUT, f.replace(f"_{a}_", f"_{b}_")))
            print(json.dumps({"file": f, "bit_equal": bool(np.array_equal(A, Bv)),
                              "max_abs_diff": float(np.abs(A - Bv).max())}))
    sys.exit(0)
import torch
from trajectory_generator_ros2_amd.solver import Solver
from trajectory_generator_ros2_amd import METHOD_DENSE_KKT, synthetic as S
tag = os.environ.get("KB_TAG", "default")
B = int(os.environ.get("KB_B", 16384)); K = 5
s = Solver(0)
for M in [int(m) for m in os.environ.get("KB_MS", "3,10").split(",")]:
    _, W, T = S.uniform_batch(B, M)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda"); dR = torch.empty_like(dC)
    dS = torch.empty((B,), dtype=torch.int32, device="cuda")
    s.set_method(0)
    s.solve_uniform_device(B, M, dW, dT, dR, dS)
    s.set_method(METHOD_DENSE_KKT)
    s.solve_uniform_device(B, M, dW, dT, dC, dS)
    torch.cuda.synchronize()
    ts = []
    for _ in range(K):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); s.solve_uniform_device(B, M, dW, dT, dC, dS); e1.record()
        torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    err = ((dC - dR).abs().amax(dim=(1, 3)) / dR.abs().amax(dim=(1, 3))).max().item()
    np.save(os.path.join(OUT, f"dense_{tag}_M{M}.npy"), dC.cpu().numpy())
    print(json.dumps({"tag": tag, "B": B, "M": M, "median_ms": sorted(ts)[K // 2],
                      "ms_per_65536": sorted(ts)[K // 2] * 65536 / B, "max_rel_diff_vs_reduced": err,
                      "status_ok": bool((dS == 0).all().item())}), flush=True)
