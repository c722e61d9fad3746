#!/usr/bin/env python3
"""Headline workload (config 3: 65,536 x M = 10, a fresh batch every launch, 4 sets rotated):
does running consecutive, independent batches on two streams (one handle each) overlap
one launch's input loads and factorisation with the previous launch's store drain?
K launches per mode, timed with events around the whole sequence (both streams joined):
  one      one stream, one handle, direct launches (the bench's order without its graph)
  two      launches alternate between two streams / two handles, direct launches
  graph1   one stream captured into one HIP graph (the bench's mode)
  graph2   two streams captured into one HIP graph (fork / join), launches alternating
One JSON line: us per launch for each mode."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from trajectory_generator_ros2_amd import synthetic as S
from trajectory_generator_ros2_amd.solver import Solver

B, M, SETS = 65536, 10, 4
K = int(os.environ.get("OV_K", "60"))
dev = torch.device("cuda", 0)
bufs = []
for k in range(SETS):
    _, W, T = S.uniform_batch(B, M, seed=S.SEED + k)
    bufs.append((torch.from_numpy(W.reshape(-1, 3).copy()).to(dev), torch.from_numpy(T.reshape(-1).copy()).to(dev),
                 torch.empty((B * M, 3, 8), dtype=torch.float64, device=dev),
                 torch.empty((B,), dtype=torch.int32, device=dev)))
solvers = [Solver(0), Solver(0)]
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def launch(k, nstreams):
    i = k % nstreams
    dW, dT, dC, dS = bufs[k % SETS]
    solvers[i].solve_uniform_device(B, M, dW, dT, dC, dS, stream=streams[i].cuda_stream)


def run_direct(nstreams):
    main = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(main)
    for s in streams[:nstreams]:
        s.wait_stream(main)
    for k in range(K):
        launch(k, nstreams)
    for s in streams[:nstreams]:
        main.wait_stream(s)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


def capture(nstreams):
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
        for s in streams[:nstreams]:
            s.wait_stream(cap)
        for k in range(K):
            launch(k, nstreams)
        for s in streams[:nstreams]:
            cap.wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    return g


def run_graph(g):
    main = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(main)
    g.replay()
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


for n in (1, 2):  # warm both handles and streams
    run_direct(n)
graphs = {}
for n in (1, 2):
    try:
        graphs[n] = capture(n)
    except Exception as e:  # report, keep the direct modes
        graphs[n] = None
        print(f"capture with {n} streams failed: {e}", file=sys.stderr)
res = {"one": [], "two": [], "graph1": [], "graph2": []}
for rep in range(5):
    res["one"].append(run_direct(1))
    res["two"].append(run_direct(2))
    if graphs[1] is not None:
        res["graph1"].append(run_graph(graphs[1]))
    if graphs[2] is not None:
        res["graph2"].append(run_graph(graphs[2]))
for dS in (b[3] for b in bufs):
    assert int((dS != 0).sum()) == 0
out = {k: {"median_us": float(np.median(v)), "min_us": float(np.min(v))} for k, v in res.items() if v}
out["K"] = K
out["B"], out["M"] = B, M
print(json.dumps(out))
