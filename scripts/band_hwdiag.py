#!/usr/bin/env python3
"""Band-KKT diagnosis with a TGMS_BAND_HWID build (TGMS_LIB): the status word of every
trajectory carries where it ran (HW_ID bits 0..19: wave slot, SIMD, CU, SH, SE, workgroup
slot on the CU; bits 20..23 the XCC; bits 24..27 the real status).  Compares the band
solve with the reduced solve and prints, for the wrong trajectories, histograms over
each placement field next to the same histogram over all trajectories."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import METHOD_BAND_KKT, synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B = int(os.environ.get("KB_B", 131072)); M = int(os.environ.get("KB_M", 16))
REPS = int(os.environ.get("KB_REPS", 2))
_, W, T = S.uniform_batch(B, M, seed=int(os.environ.get("KB_SEED", 7000)))
dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda"); dR = torch.empty_like(dC)
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
s = Solver(0)
s.solve_uniform_device(B, M, dW, dT, dR, dS)
s.set_method(METHOD_BAND_KKT)
fields = {"wave": (0, 4), "simd": (4, 2), "cu": (8, 4), "sh": (12, 1), "se": (13, 3), "tg": (16, 4),
          "xcc": (20, 4), "st": (24, 4)}
for rep in range(REPS):
    dC.zero_()
    s.solve_uniform_device(B, M, dW, dT, dC, dS)
    torch.cuda.synchronize()
    err = ((dC - dR).abs().amax(dim=(1, 3)) / dR.abs().amax(dim=(1, 3))).amax(dim=1).cpu().numpy()
    hw = dS.cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    bad = np.nonzero(err > 1e-9)[0]
    out = {"rep": rep, "B": B, "M": M, "n_bad": int(bad.size), "slots": np.bincount(bad % 16, minlength=16).tolist(),
           "bad_zero": int((dC[torch.from_numpy(bad).cuda()].abs().amax(dim=(1, 2, 3)) == 0).sum().item()) if bad.size else 0,
           "max_err": float(err.max())}
    for f, (o, w) in fields.items():
        v = (hw >> o) & ((1 << w) - 1)
        n = 1 << w
        out[f] = {"all": np.bincount(v, minlength=n).tolist(), "bad": np.bincount(v[bad], minlength=n).tolist()}
    # distinct (xcc, se, sh, cu) places and how many workgroup slots each used
    place = (hw >> 8) & 0xFF | (((hw >> 20) & 0xF) << 8)  # CU, SH, SE, XCC (not the workgroup slot)
    tg = (hw >> 16) & 0xF
    pt = np.unique(place * 16 + tg)
    cnt = np.bincount(pt // 16)
    out["cus_used"] = int((cnt > 0).sum()); out["cus_with_2plus_tg"] = int((cnt > 1).sum())
    if bad.size:
        out["bad_places"] = int(np.unique(place[bad]).size)
        out["bad_first"] = bad[:8].tolist()
        out["bad_group_round"] = np.bincount(bad // 16 // 1024).tolist()
    print(json.dumps(out), flush=True)
