#!/usr/bin/env python3
"""Config 5, one GPU's share (bench.py's config5 line: shard 0 of 8 of the 1,048,576
ragged batch, M ~ U{2..16}): K calls of tgms_refine_loop_device (10 steps + cost +
final solve), timed with HIP events around each call on the launch stream (GPU time)
and by wall clock (host planning included).  C5_B overrides the global batch size; C5_MSEL=lo-hi keeps only the shard's trajectories
with lo <= M <= hi (one occupancy class timed alone on the same trajectories)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import shard as SH
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

K = int(os.environ.get("C5_K", "10"))
Bt = int(os.environ.get("C5_B", "1048576"))
so_all, W_all, T_all = S.ragged_batch(Bt, 2, 16)
bounds = SH.ragged_bounds(so_all, 8)
so, W, T, _ = SH.shard_csr(so_all, W_all, T_all, None, int(bounds[0]), int(bounds[1]))
so = so.astype(np.int32)
if os.environ.get("C5_MSEL"):  # "lo-hi": keep only this shard's trajectories with lo <= M <= hi
    mlo, mhi = (int(x) for x in os.environ["C5_MSEL"].split("-"))
    Ms = np.diff(so)
    keep = np.nonzero((Ms >= mlo) & (Ms <= mhi))[0]
    Wr = np.asarray(W).reshape(-1, 3)
    W = np.concatenate([Wr[so[i] + i:so[i + 1] + i + 1] for i in keep])
    T = np.concatenate([T[so[i]:so[i + 1]] for i in keep])
    so = np.concatenate([[0], np.cumsum(Ms[keep])]).astype(np.int32)
B = len(so) - 1
s = Solver(0)
d_so = torch.from_numpy(so).cuda()
dW = torch.from_numpy(np.ascontiguousarray(W).reshape(-1, 3)).cuda()
T0 = torch.from_numpy(np.ascontiguousarray(T).reshape(-1)).cuda()
dT = torch.empty_like(T0)
dC = torch.empty((int(so[-1]), 3, 8), dtype=torch.float64, device="cuda")
dcost = torch.empty(B, dtype=torch.float64, device="cuda")
dst = torch.empty(B, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
sp = st.cuda_stream
for _ in range(3):
    dT.copy_(T0)
    s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=sp)
torch.cuda.synchronize()
evs = []
for _ in range(K):
    dT.copy_(T0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=sp)
    e1.record(st)
    evs.append((e0, e1))
torch.cuda.synchronize()
ev_ms = sorted(a.elapsed_time(b) for a, b in evs)
# K calls back to back between ONE event pair (no copies between: the times keep refining,
# the work per call is the same): per-call GPU time including the per-call stream packets
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(K):
    s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=sp)
e1.record(st)
torch.cuda.synchronize()
b2b = e0.elapsed_time(e1) / K
t0 = time.perf_counter()
for _ in range(K):
    dT.copy_(T0)
    s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=sp)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / K * 1e3
t0 = time.perf_counter()
for _ in range(K):  # host cost of one call (planning + graph launch), GPU idle-waiting
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    s.refine_loop_device(so, d_so, dW, dT, 1.0, 0.1, 10, dC, dcost, dst, stream=sp)
    hh = time.perf_counter() - h0
torch.cuda.synchronize()
assert int((dst != 0).sum()) == 0
print(json.dumps({"B": B, "segments": int(so[-1]), "ms_events_median": ev_ms[K // 2], "ms_events_min": ev_ms[0], "ms_back_to_back": b2b,
                  "ms_wall_per_call": wall, "host_ms_last_call": hh * 1e3,
                  "lib": os.path.basename(os.environ.get("TGMS_LIB", "default"))}))
