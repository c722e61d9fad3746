#!/usr/bin/env python3
"""Config 4 at full size (1,048,576 x M = 10) through tgms_solve_batch_multi_device on
one device (in place), and the same batch through tgms_solve_uniform_device, K calls
each, HIP events per call (for rocprofv3 kernel traces of the 2 GB output case)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B, M, K = int(os.environ.get("C4_B", "1048576")), 10, int(os.environ.get("C4_K", "5"))
so, W, T = S.uniform_batch(B, M)
dso = torch.from_numpy(so).cuda()
dW = torch.from_numpy(W.reshape(-1, 3)).cuda()
dT = torch.from_numpy(T.reshape(-1)).cuda()
dC = torch.empty((B * M, 3, 8), dtype=torch.float64, device="cuda")
dS = torch.empty((B,), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
s1 = Solver(0)
mh = Solver(device_count=1)
res = {"B": B}
for name, fn in (("uniform_device", lambda: s1.solve_uniform_device(B, M, dW, dT, dC, dS, stream=st.cuda_stream)),
                 ("batch_device", lambda: s1.solve_batch_device(so, dso, dW, dT, dC, dS, stream=st.cuda_stream)),
                 ("multi_device", lambda: mh.solve_batch_multi_device(so, dso, dW, dT, dC, dS, stream=st.cuda_stream))):
    fn()
    torch.cuda.synchronize()
    ev = []
    for _ in range(K):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        ev.append((e0, e1))
    torch.cuda.synchronize()
    res[name + "_ms"] = sorted(a.elapsed_time(b) for a, b in ev)[K // 2]
print(json.dumps(res))
