#!/usr/bin/env python3
"""Headline benchmark: min-snap trajectories/sec (10-seg, order-7, 3-axis) at batch = 65k.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one solve of one batch of B = 65,536 synthetic trajectories (M = 10)
per GPU (BASELINE.json configs[2] / SURVEY.md §8(d) config 3), inputs resident in
HBM when the timed region starts, coefficients written to HBM.  Every step solves a
FRESH batch: the K steps rotate over `--sets` (4) independent batches, 594 MB per
GPU, so no step finds its inputs or its output lines in the 256 MiB Infinity Cache
where the step before left them (the same-batch loop, whose 148.6 MB stay on-die, is
reported beside it as `cache_resident`).  Trajectories are independent, so N GPUs
each solve their own shard (weak scaling, no data-path collective).  Rank 0 prints
ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6   # MI355X FP64 vector spec peak (dense-KKT roof, reported beside)


def algorithmic_bytes_per_traj(M: int, with_status: bool = True) -> int:
    """input (M+1)*3*8 waypoints + M*8 times, output M*3*8*8 coefficients
    (+ 4 B status).  M = 10: 264 + 80 + 1920 (+4) bytes."""
    return (M + 1) * 3 * 8 + M * 8 + M * 24 * 8 + (4 if with_status else 0)


def band_flops_per_traj(M: int) -> float:
    """GEPP flops that touch the band of the interleaved KKT (kl = 9, U width 19) with
    3 right-hand sides: per column 9 multipliers + 9 x (18 + 3) updates, then back
    substitution over 18 super-diagonals x 3 axes."""
    N = 14 * M + 2
    return N * (9 + 2 * 9 * 21) + N * 3 * 2 * 18


def refine_flops_per_traj(M: int, iters: int = 10) -> float:
    """Algorithmic FP64 flops of one config-5 call per trajectory: the
    one-sided block LDL^T of DESIGN.md §2 over the M - 1 interior knots, three axes, counted
    operation by operation (an FMA is 2 flops; a reciprocal 1), `iters` passes that end in the
    cost and its T-derivative per segment-axis plus the update, and one pass that ends in the
    coefficients and the cost (seg_cost_q).  Per interior knot: powers 6, the diagonal block
    18, the coupling 9, G = S^-1 C 45 and the Schur update 36 (from the second knot on), the
    3x3 LDL^T 14; per knot and axis: right-hand side 11, forward 33, back 18.  Per segment and
    axis in a gradient pass (round 6: the Legendre-basis form, seg_grad_u): the scaled end
    data 6, cost and gradient 44, accumulation 4 (round 5's count, for the P4..P7 form it
    replaced: 58 + 84); in the last pass the Hermite -> P4..P7 map 58, the coefficients 4 and
    the cost 27; per segment the powers r^2, r^3 2 and the update 8.  This is what the
    algorithm needs, not what the lane-pair kernels execute (their twisted interface and
    duplicated blocks are in the executed count beside it)."""
    nk = M - 1
    fac = nk * (6 + 18 + 9 + 14) + max(nk - 1, 0) * (45 + 36)
    sub = 3 * (nk * (11 + 18) + nk * 15 + max(nk - 1, 0) * 18)
    grad_pass = fac + sub + M * 3 * (6 + 44 + 4) + M * (2 + 8)
    final_pass = fac + sub + M * 3 * (58 + 4 + 27)
    return float(iters * grad_pass + final_pass)


def dense_flops_per_traj(M: int) -> float:
    N = 14 * M + 2
    return 2.0 / 3.0 * N ** 3 + 6.0 * N ** 2


TRAFFIC_FILE = "profiles/pmc_traffic.json"


def load_traffic(workload_key: str):
    """Per-launch HBM bytes of this workload from the committed rocprofv3 PMC passes
    (scripts/gpu_profile.sh -> scripts/pmc_traffic.py -> profiles/pmc_traffic.json):
    PMC counters cannot be read inside this process, so the line reports the
    committed measurement of the same command and names its source.  None if absent."""
    try:
        with open(os.path.join(ROOT, TRAFFIC_FILE)) as f:
            d = json.load(f)
        e = d.get(workload_key)
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def available_cores() -> dict:
    """Host cores this process may use: the affinity mask, capped by the cgroup CPU
    quota (a container's share of a larger machine), as used by the CPU baseline."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cgroup_quota": quota, "usable": min(aff, quota) if quota else aff}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _timed_reps(fn, n_per_call: int, target_s: float):
    """Repeat fn() until about target_s of work is done; returns (items/s, reps, seconds)."""
    t0 = time.perf_counter()
    fn()
    pilot = max(time.perf_counter() - t0, 1e-6)
    reps = max(1, int(round(target_s / pilot)))
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    el = time.perf_counter() - t0
    return n_per_call * reps / el, reps, el


def cpu_baseline(B: int, M: int, target_s: float, check=None):
    """CPU restatement of the solve (the reference has no solver to time, SURVEY.md §0,
    §8(d)): the oracle's fp64 C code with OpenMP over trajectories, on every core this
    process may use, on a bounded sample of the same workload.  `value` is its reduced
    formulation (the GPU kernel's math, O(M) per trajectory: the strongest CPU
    restatement); the survey's literal dense-KKT LU and the one-core rates are beside it.

    The timed sample is rank 0's batch 0 (seed 20251015), the batch the headline's steps
    k = 0 mod sets solved: `check` ([B', 3, 8], what the timed region wrote for its first B'
    trajectories) is compared with the baseline's own last output, norm-wise per
    (trajectory, axis), outside every timed region.  Returns (line, check result)."""
    from oracle import oracle as O
    from trajectory_generator_ros2_amd import synthetic as S
    O.build()
    cores = available_cores()
    threads = cores["usable"]
    so, W, T = S.uniform_batch(B, M)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    last = {}

    def reduced():
        last["C"], st = O.solve_batch(so, W, T, None, O.REDUCED, threads)
        assert (st == 0).all()

    red_rate, red_reps, red_s = _timed_reps(reduced, B, 0.6 * target_s)
    # dense KKT on a prefix sized to ~0.4 target_s
    n = 4096
    so_n = so[: n + 1]

    def dense():
        _, st = O.solve_batch(so_n, W[: n * (M + 1)], T[: n * M], None, O.KKT_C4, threads)
        assert (st == 0).all()

    dense_rate, dense_reps, dense_s = _timed_reps(dense, n, 0.4 * target_s)
    t1 = time.perf_counter()
    O.solve_batch(so[:8193], W[: 8192 * (M + 1)], T[: 8192 * M], None, O.REDUCED, 1)
    red_1 = 8192 / (time.perf_counter() - t1)
    t1 = time.perf_counter()
    O.solve_batch(so[:1025], W[: 1024 * (M + 1)], T[: 1024 * M], None, O.KKT_C4, 1)
    dense_1 = 1024 / (time.perf_counter() - t1)
    res = None
    if check is not None:
        n = check.shape[0] // M
        R = last["C"][: n * M].reshape(n, M, 3, 8)
        G = check.reshape(n, M, 3, 8)
        den = np.abs(R).max(axis=(1, 3))
        err = np.abs(G - R).max(axis=(1, 3)) / np.where(den == 0.0, 1.0, den)
        res = {"trajectories": n, "max_rel_err": float(err.max()), "tol": 1e-9,
               "ok": bool(np.isfinite(G).all() and err.max() <= 1e-9)}
    return {"value": red_rate, "unit": "trajectories/s", "cores": threads, "kind": "cpu_restatement",
            "what": "cpu_restatement (reference has no solver): oracle/minsnap_oracle.c, fp64, OpenMP",
            "cores_detail": cores, "cpu_model": _cpu_model(),
            "value_1core": red_1, "dense_kkt_value": dense_rate, "dense_kkt_value_1core": dense_1,
            "sample": f"reduced formulation: {red_reps} x {B} trajectories of the config-3 workload (M={M}), "
                      f"{red_s:.1f} s; dense KKT (LU, partial pivoting): {dense_reps} x {n}, {dense_s:.1f} s; "
                      f"{threads} OpenMP thread(s)"}, res


C5_PMC_FILE = "profiles/c5_pmc.json"
BYTE_MIX_FLOOR_US = 28.6  # config 3's byte mix with no compute, best occupancy (profiles/archive/r03_runstore_occ.txt;
#                            round 6 on another box: 29.1 us, profiles/r06_floor.jsonl -- the lower one is kept)
# the same bytes with consecutive launches overlapping over 4 streams in one graph, best occupancy
# (scripts/micro/floor.hip, profiles/r06_floor.jsonl): the floor of the headline's pipelined region
PIPELINED_FLOOR_US = 27.4


def _c5_shard(so_all, W_all, T_all, bounds, part, dev):
    """Shard `part` of the config-5 batch, resident on `dev`."""
    import torch
    from trajectory_generator_ros2_amd import shard as SH
    so, W, T, _ = SH.shard_csr(so_all, W_all, T_all, None, int(bounds[part]), int(bounds[part + 1]))
    B = len(so) - 1
    Sg = int(so[-1])
    return {"so": so, "B": B, "Sg": Sg, "d_so": torch.from_numpy(so.astype(np.int32)).to(dev),
            "dW": torch.from_numpy(W.reshape(-1, 3)).to(dev), "T0": torch.from_numpy(T.reshape(-1)).to(dev)}


def _c5_time(solver, sh, dev, stream, iters, k_T, eta, reps):
    """Median HIP-event time of one tgms_refine_loop_device call over shard `sh` (times
    reset from a device copy before each call, outside the events), the wall time per
    call, and the statuses of the last call."""
    import torch
    so, B, Sg = sh["so"], sh["B"], sh["Sg"]
    dT = torch.empty_like(sh["T0"])
    dC = torch.empty((Sg, 3, 8), dtype=torch.float64, device=dev)
    dcost = torch.empty(B, dtype=torch.float64, device=dev)
    dst = torch.empty(B, dtype=torch.int32, device=dev)
    sp = stream.cuda_stream

    def call():
        solver.refine_loop_device(so, sh["d_so"], sh["dW"], dT, k_T, eta, iters, dC, dcost, dst, stream=sp)

    for _ in range(2):
        dT.copy_(sh["T0"])
        call()
    torch.cuda.synchronize()
    evs = []
    for _ in range(reps):
        dT.copy_(sh["T0"])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        call()
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]
    t0 = time.perf_counter()
    for _ in range(reps):
        dT.copy_(sh["T0"])
        call()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    host = []
    for _ in range(reps):  # host time of one call (scan + graph replay), the GPU idle
        dT.copy_(sh["T0"])
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        call()
        host.append((time.perf_counter() - h0) * 1e3)
        torch.cuda.synchronize()
    _c5_time.host_ms = sorted(host)[reps // 2]
    return ms, wall, int((dst != 0).sum().item())


def config5_line(solver, dev, stream, world, rank, B_total=1048576, iters=10, k_T=1.0, eta=0.1, reps=5):
    """Config 5: a 1,048,576-trajectory ragged batch (M ~ U{2..16}) split over 8 GPUs
    (the configuration's count, whatever N is) into contiguous cost-balanced shards
    (shard.ragged_bounds); this rank solves shard `rank % 8`: `iters` time-refinement
    steps + the final solve, one tgms_refine_loop_device call (planned once).
    `ms_per_batch` is the median of HIP-event pairs around single calls on the launch
    stream (the times are reset from a device copy before each call, outside the
    events); the wall clock per call (host planning included) is beside it.

    Shard balance: at N = 1 every one of the 8 shards is timed the
    same way on this GPU, one after another; `shard_balance` = max / mean of those times
    (at N = 8 the config-5 time is the slowest shard's).

    Roofline: the loop is FP64-VALU-bound.  `achieved` = the executed FP64 flops of one
    call (committed PMC, profiles/c5_pmc.json) / the live event time, against the FP64
    vector peak; the algorithmic HBM bytes (waypoints + times read, times + coefficients
    + costs + statuses written) and their rate are beside it."""
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    so_all, W_all, T_all = S.ragged_batch(B_total, 2, 16)
    bounds = SH.ragged_bounds(so_all, 8)
    part = rank % 8
    sh = _c5_shard(so_all, W_all, T_all, bounds, part, dev)
    B, Sg = sh["B"], sh["Sg"]
    ms, wall, bad = _c5_time(solver, sh, dev, stream, iters, k_T, eta, reps)
    assert bad == 0, "refinement reported failures"
    shard_ms = None
    if world == 1:
        shard_ms = []
        for p in range(8):
            shp = sh if p == part else _c5_shard(so_all, W_all, T_all, bounds, p, dev)
            m_p, _, bad = _c5_time(solver, shp, dev, stream, iters, k_T, eta, 3)
            assert bad == 0, "refinement reported failures"
            shard_ms.append(m_p)
            del shp
    del so_all, W_all, T_all
    nbytes = (Sg + B) * 24 + 2 * Sg * 8 + Sg * 192 + B * (8 + 4) + (B + 1) * 4
    line = {"workload": f"config5: shard {part} of 8 (cost-balanced, {B} trajectories) of a {B_total}-trajectory "
                        f"ragged batch, M~U{{2..16}}, {iters} refinement steps + final solve",
            "ms_per_batch": ms, "ms_wall_per_call": wall, "host_ms_per_call": getattr(_c5_time, "host_ms", None),
            "trajectories_per_s": B / (ms * 1e-3), "segments": Sg,
            "k_T": k_T, "eta": eta,
            "timing": "median of single-call HIP event pairs on the launch stream; wall per call beside"}
    if shard_ms:
        line["shard_ms"] = shard_ms
        line["shard_balance"] = max(shard_ms) / (sum(shard_ms) / len(shard_ms))
        line["shard_sizes"] = np.diff(bounds).tolist()
    try:
        pmc = json.load(open(os.path.join(ROOT, C5_PMC_FILE)))["c5_share"]
    except (OSError, ValueError, KeyError):
        pmc = None
    hbm = {"algorithmic_bytes_per_call": nbytes, "achieved_GBs": nbytes / (ms * 1e-3) / 1e9,
           "frac_of_peak": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "traffic": pmc["hbm_bytes_per_call"] if pmc else None}
    # lane-accurate restatement: the PMC counts every executed FP64
    # wave-instruction as 64 lanes, but a group of n trajectories of one M runs in
    # ceil(n / 32) lane-pair wavefronts, so its last wavefront is partly idle.  Weighting
    # each M group's wavefronts by its work per wavefront (~ 2 + M, the planner's cost)
    # gives the fraction of executed lane-flops that belong to live trajectories.
    counts = np.bincount(np.diff(sh["so"]), minlength=17)
    w_all = w_live = 0.0
    for m_, n_ in enumerate(counts):
        if m_ == 0 or n_ == 0:
            continue
        waves = -(-int(n_) // 32)
        w_all += waves * (2 + m_)
        w_live += waves * (2 + m_) * (2.0 * n_ / (64.0 * waves))
    lane_frac = w_live / w_all if w_all else 1.0
    m_of = np.diff(sh["so"])
    alg_flops = float(sum(refine_flops_per_traj(int(m_), iters) * int(c_)
                          for m_, c_ in enumerate(np.bincount(m_of, minlength=17)) if m_ and c_))
    tf_alg = alg_flops / (ms * 1e-3) / 1e12
    if pmc:
        tf = pmc["fp64_flops_per_call"] / (ms * 1e-3) / 1e12
        tf_lane = tf * lane_frac
        line["roofline"] = {"bound": "fp64_valu", "achieved": tf_alg, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                            "frac": tf_alg / FP64_PEAK_TFS, "flops_per_call": alg_flops,
                            "flops_definition": "algorithmic: bench.refine_flops_per_traj (the O(M) block LDL^T, "
                                                "gradient and update, operation by operation) summed over the shard",
                            "lane_fraction": lane_frac,
                            "executed_lane_accurate": {"achieved": tf_lane, "frac": tf_lane / FP64_PEAK_TFS,
                                                       "flops_per_call": pmc["fp64_flops_per_call"] * lane_frac},
                            "executed": {"achieved": tf, "frac": tf / FP64_PEAK_TFS,
                                         "flops_per_call": pmc["fp64_flops_per_call"],
                                         "note": "every executed FP64 wave-instruction counted as 64 lanes"},
                            "flops_source": f"{C5_PMC_FILE} (executed FP64 flops, rocprofv3 --pmc of "
                                            f"scripts/c5bench.py: the same call), / this run's event time",
                            "valu_issue_frac": pmc["valu_insts_per_call"] * 4 / (1024 * 2.4e9 * ms * 1e-3),
                            "hbm": hbm, "kernels": "k_refine_loop_dev<1,13> (two waves per SIMD) + <14,16> (one), concurrent"}
    else:
        line["roofline"] = {"bound": "fp64_valu", "achieved": tf_alg, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                            "frac": tf_alg / FP64_PEAK_TFS, "flops_per_call": alg_flops, "hbm": hbm}
    return line


def config4_line(solver, M, dev, stream, world, rank, B=131072, chunks=8, reps=3):
    """Config 4 (1,048,576 goals over 8 GPUs): every rank solves its 131,072-trajectory
    shard (seed + rank) and the coefficients are gathered to rank 0 over RCCL, piece by
    piece while the next piece is solved (shard.pipelined_gather).  Also reports the
    solve alone at this size: 297 MB per launch, beyond the 256 MB Infinity Cache, so
    it is the HBM-resident rate of the kernel.  At N = 1 there is nothing to gather."""
    import torch
    import torch.distributed as dist
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    _, W, T = S.uniform_batch(B, M, seed=S.SEED + rank)
    dW = torch.from_numpy(W).to(dev)
    dT = torch.from_numpy(T).to(dev)
    dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device=dev)
    dS = torch.zeros((B,), dtype=torch.int32, device=dev)
    sp = stream.cuda_stream

    def solve_chunk(lo, hi):
        solver.solve_uniform_device(hi - lo, M, dW[lo:hi], dT[lo:hi], dC[lo:hi], dS[lo:hi], stream=sp)

    # solve alone (kernel rate beyond the Infinity Cache)
    solve_chunk(0, B)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        solve_chunk(0, B)
    e1.record(stream)
    torch.cuda.synchronize()
    solve_ms = e0.elapsed_time(e1) / reps
    assert int((dS != 0).sum().item()) == 0, "solver reported failures"
    line = {"workload": f"config4: {B} trajectories/GPU x {M} segments ({world * B} total), "
                        f"coefficients gathered to rank 0",
            "solve_ms": solve_ms,
            "solve_GBs": algorithmic_bytes_per_traj(M) * B / (solve_ms * 1e-3) / 1e9}
    if world == 1:
        line["gather"] = None
        return line

    out = torch.empty((world, B, M, 3, 8), dtype=torch.float64, device=dev) if rank == 0 else None

    def run():
        for w in SH.pipelined_gather(solve_chunk, dC, chunks, dst=0, out=out):
            w.wait()
        torch.cuda.synchronize()

    run()
    ts = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ts.append(float(t.item()))
    ms = sorted(ts)[len(ts) // 2] * 1e3
    if rank == 0:
        # the gathered shards are the other ranks' solves: re-solve a slice of each
        # rank's inputs here and compare bit for bit (same kernel, same inputs)
        n = 1024
        chk = torch.empty((n, M, 3, 8), dtype=torch.float64, device=dev)
        for r in range(world):
            _, Wr, Tr = S.uniform_batch(B, M, seed=S.SEED + r)
            solver.solve_uniform_device(n, M, torch.from_numpy(Wr[:n]).to(dev), torch.from_numpy(Tr[:n]).to(dev),
                                        chk, None, stream=sp)
            torch.cuda.synchronize()
            assert torch.equal(chk, out[r, :n]), f"gathered shard of rank {r} differs"
    gathered = (world - 1) * B * M * 24 * 8
    backend = dist.get_backend()
    line["gather"] = {"collective": f"torch.distributed.gather per piece, overlapped with the solve (backend {backend}"
                                    + (": RCCL send/recv)" if backend == "nccl" else ")"),
                      "pieces": chunks, "ms_total": ms, "trajectories_per_s": world * B / (ms * 1e-3),
                      "bytes_into_rank0": gathered, "rank0_ingest_GBs": gathered / (ms * 1e-3) / 1e9}
    return line


def launch_stats(solver, B, M, bufs, stream, warm=3, n=25):
    """SURVEY.md §8(d) timing method, kernel only: `warm` untimed launches, then `n`
    launches each bracketed by its own pair of HIP events on the launch stream, a fresh
    batch every launch (the sets rotated as in the headline); median and spread."""
    import torch
    sp = stream.cuda_stream
    sets = len(bufs)
    for k in range(warm):
        dW, dT, dC, dS = bufs[k % sets]
        solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for k in range(n):
        dW, dT, dC, dS = bufs[(warm + k) % sets]
        ev[k][0].record(stream)
        solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    q = lambda f: us[min(n - 1, int(f * n))]
    return {"launches": n, "warmup": warm, "median_us": q(0.5), "p10_us": q(0.1), "p90_us": q(0.9),
            "min_us": us[0], "max_us": us[-1],
            "median_GBs": algorithmic_bytes_per_traj(M) * B / (q(0.5) * 1e-6) / 1e9,
            "how": "one HIP event pair per launch on the launch stream, a fresh batch every launch"}


def cache_resident_line(solver, B, M, buf, stream, K=40):
    """The same launch re-solving ONE batch K times: its 148.6 MB (inputs + output)
    stay in the 256 MiB Infinity Cache between launches, so the coefficient stores
    merge on-die.  A kernel-benchmark figure, reported beside the headline (which
    rotates over fresh batches), never as it."""
    import torch
    dW, dT, dC, dS = buf
    sp = stream.cuda_stream
    solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(K):
        solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    assert int((dS != 0).sum().item()) == 0, "solver reported failures"
    gbs = algorithmic_bytes_per_traj(M) * B / (ms * 1e-3) / 1e9
    return {"working_set_MB": algorithmic_bytes_per_traj(M) * B / 1e6, "launch_ms": ms,
            "trajectories_per_s": B / (ms * 1e-3), "achieved_GBs": gbs, "frac_of_peak": gbs / HBM_PEAK_GBS}


def node_line(reps=20):
    """Config 1 through the node's own path: one goal of 4 waypoints (3 segments) from
    parameters to a sampled 100 Hz Goal stream — MinSnap::readParameters (validation +
    tgms_solve_batch, B = 1) then generateTraj (tgms_sample_batch + append), the
    calls TrajectoryGenerator makes at start-up (src/TrajectoryGenerator.cpp:54, :71).
    Beside it the CPU oracle's solve + sample of the same goal (1 core)."""
    from oracle import oracle as O
    from trajectory_generator_ros2_amd.node import MinSnapNode
    wp = [0.0, 0.0, 1.0, 2.0, 1.0, 1.5, 3.0, -1.0, 2.0, 0.5, -2.0, 1.0]
    st = [2.0, 2.0, 2.5]
    params = {"alt": 1.8, "pub_freq": 100.0, "traj_type": "MinSnap", "waypoints": wp, "seg_times": st,
              "yaw_mode": "constant", "yaw": 0.0, "stop_accel": 1.0, "x_min": -5.0, "x_max": 5.0,
              "y_min": -5.0, "y_max": 5.0, "z_min": -5.0, "z_max": 5.0}
    ts, n_goals = [], 0
    for _ in range(reps + 2):
        t0 = time.perf_counter()
        n = MinSnapNode(params)
        assert n.read_parameters()
        n_goals = n.generate_traj()
        ts.append(time.perf_counter() - t0)
        n.close()
    gpu_ms = sorted(ts[2:])[reps // 2] * 1e3
    n = MinSnapNode(params)
    assert n.read_parameters()
    n.generate_traj()
    tw = []
    for _ in range(reps):
        t0 = time.perf_counter()
        n.generate_traj()
        tw.append(time.perf_counter() - t0)
    n.close()
    W, T = np.array(wp).reshape(-1, 3), np.array(st)
    tc = []
    for _ in range(reps):
        t0 = time.perf_counter()
        R, s = O.solve(W, T)
        O.sample(R, T, W, None, 0.01)
        tc.append(time.perf_counter() - t0)
    return {"workload": "config1: 1 goal, 4 waypoints, 3 segments, sampled at 100 Hz (650 goals)",
            "goals": n_goals, "ms_params_to_goals": gpu_ms,
            "ms_generate_traj_warm": sorted(tw)[reps // 2] * 1e3,
            "cpu_oracle_ms_solve_and_sample": sorted(tc)[reps // 2] * 1e3}


def uniform_large_m_line(solver, dev, stream, Ms=(12, 14, 16), B=65536, sets=4, K=20):
    """Uniform batches above the lane kernel's M range: 65,536
    trajectories per launch, a fresh batch every launch (`sets` rotated, beyond the Infinity
    Cache), HIP events around K launches; algorithmic bytes as the headline's.  Even M >= 12
    run the joint lane-pair solve with whole-line output (k_reduced_uniform_lines)."""
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    out = {}
    sp = stream.cuda_stream
    for M in Ms:
        bufs = []
        for k in range(sets):
            _, Wk, Tk = S.uniform_batch(B, M, seed=S.SEED + 1000 + k)
            bufs.append((torch.from_numpy(Wk).to(dev), torch.from_numpy(Tk).to(dev),
                         torch.empty((B, M, 3, 8), dtype=torch.float64, device=dev)))
        dS = torch.empty(B, dtype=torch.int32, device=dev)
        for k in range(sets):
            solver.solve_uniform_device(B, M, *bufs[k], dS, stream=sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(K):
            solver.solve_uniform_device(B, M, *bufs[k % sets], dS, stream=sp)
        e1.record(stream)
        torch.cuda.synchronize()
        assert int((dS != 0).sum().item()) == 0, "solver reported failures"
        us = e0.elapsed_time(e1) / K * 1e3
        nbytes = algorithmic_bytes_per_traj(M) * B
        kern = (f"k_lane_uniform<{M}>" if M % 2 == 0 and M <= 10 else
                f"k_reduced_uniform_lines<{M}>" if M % 2 == 0 else f"k_reduced_uniform<{M}>")
        out[f"M{M}"] = {"us_per_launch": us, "algorithmic_bytes": nbytes, "GBs": nbytes / (us * 1e-6) / 1e9,
                        "frac": nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, "kernel": kern}
        del bufs
        torch.cuda.empty_cache()
    out["workload"] = f"uniform {B} x M in {list(Ms)}, fresh batch every launch ({sets} rotated), events over {K}"
    return out


def host_backend_node_line(reps=20):
    """Config 1 as BASELINE.json states it, "ROS2 node up, no GPU": the node's MinSnap
    primitive on the explicit host backend (`minsnap_backend: host`, tgms_create_host) --
    readParameters (validation + solve, B = 1) and generateTraj (sample + append) on this
    CPU thread, as the reference generates on its executor thread."""
    from trajectory_generator_ros2_amd.node import MinSnapNode
    wp = [0.0, 0.0, 1.0, 2.0, 1.0, 1.5, 3.0, -1.0, 2.0, 0.5, -2.0, 1.0]
    params = {"alt": 1.8, "pub_freq": 100.0, "traj_type": "MinSnap", "waypoints": wp, "seg_times": [2.0, 2.0, 2.5],
              "yaw_mode": "constant", "yaw": 0.0, "stop_accel": 1.0, "x_min": -5.0, "x_max": 5.0,
              "y_min": -5.0, "y_max": 5.0, "z_min": -5.0, "z_max": 5.0, "minsnap_backend": "host"}
    ts, n_goals = [], 0
    for _ in range(reps + 2):
        t0 = time.perf_counter()
        n = MinSnapNode(params)
        assert n.read_parameters()
        n_goals = n.generate_traj()
        ts.append(time.perf_counter() - t0)
        n.close()
    return {"workload": "config1 on the host backend (no GPU used): 1 goal, 4 waypoints, 3 segments, 100 Hz",
            "goals": n_goals, "ms_params_to_goals": sorted(ts[2:])[reps // 2] * 1e3, "cores": 1}


def host_line(solver, B, M, W, T, reps=20):
    """PCIe-inclusive rate: tgms_solve_batch on host buffers (H2D, solve, D2H), the call
    the node makes; reported beside `value`, never as it (SURVEY.md 8(d) timing)."""
    import numpy as np
    so = (np.arange(B + 1, dtype=np.int32) * M)
    Wf, Tf = W.reshape(-1, 3), T.reshape(-1)
    out = (np.zeros((B * M, 3, 8)), np.zeros(B, dtype=np.int32))  # caller-owned, reused
    for _ in range(3):  # warm-up (workspace, page faults)
        C, st, worst = solver.solve(so, Wf, Tf, out=out)
    assert worst == 0, worst
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        C, st, worst = solver.solve(so, Wf, Tf, out=out)
        ts.append(time.perf_counter() - t0)
    ms = sorted(ts)[len(ts) // 2] * 1e3
    nbytes = algorithmic_bytes_per_traj(M) * B + (B + 1) * 4
    return {"trajectories": B, "ms_per_call": ms, "ms_min": sorted(ts)[0] * 1e3, "calls": reps, "warmup": 3,
            "trajectories_per_s": B / (ms * 1e-3),
            "pcie_bytes": nbytes, "effective_GBs": nbytes / (ms * 1e-3) / 1e9,
            "path": "tgms_solve_batch (end to end: H2D, solve, D2H), pageable host numpy buffers reused across "
                    "calls; median of the calls"}


def config2_line(solver, dev, stream, reps=200, B=1024, M=3):
    """Config 2 (BASELINE configs[1]): a batch of 1,024 random 4-waypoint goals (M = 3), fp64,
    one MI355X.  1,024 trajectories are 32 lane-pair wavefronts: the call is launch- and
    latency-bound, not HBM-bound, so this line reports times, not a roofline:
      - `device_us`: HIP events over `reps` back-to-back launches on device buffers;
      - `sync_call_us`: one launch + stream synchronise, median wall clock per call;
      - `host_call_us`: tgms_solve_batch on host buffers (H2D, solve, D2H), median;
      - the literal KKT methods on the same batch (band LU, dense Gauss-Jordan), events;
      - the CPU oracle on the same batch, reduced formulation and dense KKT, one core;
    and the GPU coefficients of every method against the oracle's (norm-wise per
    (trajectory, axis), outside every timed region)."""
    import torch
    from oracle import oracle as O
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_DENSE_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(B, M)
    W2, T2 = np.ascontiguousarray(W.reshape(-1, 3)), np.ascontiguousarray(T.reshape(-1))
    dW, dT = torch.from_numpy(W2).to(dev), torch.from_numpy(T2).to(dev)
    dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device=dev)
    dS = torch.zeros((B,), dtype=torch.int32, device=dev)
    sp = stream.cuda_stream
    O.build()
    R, st = O.solve_batch(so, W2, T2, None, O.KKT_C4, 1)
    assert (st == 0).all()
    R = R.reshape(B, M, 3, 8)
    den = np.abs(R).max(axis=(1, 3))
    den = np.where(den == 0.0, 1.0, den)

    def err_vs_oracle():
        G = dC.cpu().numpy()
        return float((np.abs(G - R).max(axis=(1, 3)) / den).max())

    def events(n):
        solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
        e1.record(stream)
        torch.cuda.synchronize()
        assert int((dS != 0).sum().item()) == 0, "solver reported failures"
        return e0.elapsed_time(e1) / n * 1e3

    methods = {}
    for name, meth, n in (("band_kkt", METHOD_BAND_KKT, 50), ("dense_kkt", METHOD_DENSE_KKT, 50),
                          ("reduced", METHOD_REDUCED, reps)):  # reduced last: the handle's method after
        solver.set_method(meth)
        dC.fill_(float("nan"))
        us = events(n)
        methods[name] = {"device_us": us, "trajectories_per_s": B / (us * 1e-6), "max_rel_err_vs_oracle": err_vs_oracle()}
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        solver.solve_uniform_device(B, M, dW, dT, dC, dS, stream=sp)
        stream.synchronize()
        ts.append(time.perf_counter() - t0)
    sync_us = sorted(ts)[len(ts) // 2] * 1e6
    out = (np.zeros((B * M, 3, 8)), np.zeros(B, dtype=np.int32))
    for _ in range(3):
        solver.solve(so, W2, T2, out=out)
    th = []
    for _ in range(50):
        t0 = time.perf_counter()
        C, st, worst = solver.solve(so, W2, T2, out=out)
        th.append(time.perf_counter() - t0)
    assert worst == 0, worst
    host_us = sorted(th)[len(th) // 2] * 1e6
    host_err = float((np.abs(C.reshape(B, M, 3, 8) - R).max(axis=(1, 3)) / den).max())

    def cpu(form):
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            O.solve_batch(so, W2, T2, None, form, 1)
            n += 1
        return (time.perf_counter() - t0) / n * 1e6

    cpu_red, cpu_kkt = cpu(O.REDUCED), cpu(O.KKT_C4)
    worst_err = max([m["max_rel_err_vs_oracle"] for m in methods.values()] + [host_err])
    return {"workload": f"config2: {B} random 4-waypoint goals (M = {M}), fp64, rest-to-rest, one MI355X",
            "device_us": methods["reduced"]["device_us"], "sync_call_us": sync_us, "host_call_us": host_us,
            "trajectories_per_s": methods["reduced"]["trajectories_per_s"],
            "methods": methods,
            "cpu_oracle_1core_us": {"reduced": cpu_red, "dense_kkt": cpu_kkt},
            "max_rel_err_vs_oracle": worst_err, "tol": 1e-9, "verified": bool(worst_err <= 1e-9),
            "timing": f"events over {reps} launches (literal methods: 50); sync and host calls: median wall clock"}


def sampler_line(solver, n, M, W, T, dC, dev, stream, dt=0.01, reps=5):
    """Sampler on the first n solved trajectories at 100 Hz:
    Goal-layout p/v/a/j/psi/dpsi, HBM-bound by its output."""
    import torch
    from trajectory_generator_ros2_amd import YAW_VELOCITY
    from trajectory_generator_ros2_amd.solver import sample_offsets
    n = min(n, W.shape[0])
    so = np.arange(n + 1, dtype=np.int32) * M
    offs = sample_offsets(so, T[:n].reshape(-1), dt)
    d_so = torch.from_numpy(so).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    dWs = torch.from_numpy(np.ascontiguousarray(W[:n])).to(dev)
    dTs = torch.from_numpy(np.ascontiguousarray(T[:n])).to(dev)
    out = torch.empty((int(offs[-1]), 14), dtype=torch.float64, device=dev)
    sp = stream.cuda_stream

    def run():
        solver.sample_device(n, d_so, dWs, dTs, dC, dt, d_offs, out, yaw_mode=YAW_VELOCITY, stream=sp)

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = int(offs[-1]) * 14 * 8 + n * (M * 24 * 8 + M * 8 + (M + 1) * 24 + 4 + 8)
    return {"trajectories": n, "samples": int(offs[-1]), "dt": dt, "ms_per_launch": ms,
            "samples_per_s": int(offs[-1]) / (ms * 1e-3),
            "roofline": {"bound": "hbm", "achieved": nbytes / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_launch": nbytes, "kernel": "k_sample"}}


def resolve_topology(gpus: int, env: dict, visible: int):
    """How `--gpus N` maps onto processes and devices.

    * under a launcher (WORLD_SIZE in the environment, e.g. torch.distributed.run): one
      rank per GPU, and WORLD_SIZE must equal N;
    * no launcher: ONE process drives N devices (0..N-1) -- the shape of the reference's
      caller, one C++ process holding one Trajectory (TrajectoryGenerator.hpp:83) --
      and N must not exceed the visible devices.
    Returns ("ranks", world, rank, local) or ("process", N, 0, 0); raises SystemExit
    with a message otherwise."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: launched with WORLD_SIZE={world} ranks but --gpus {gpus}; "
                             f"start one rank per GPU (--nproc-per-node {gpus}) or drop the launcher")
        return "ranks", world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))
    if gpus > visible:
        raise SystemExit(f"bench.py: --gpus {gpus} but only {visible} HIP device(s) are visible; "
                         f"refusing to report a {gpus}-GPU line from fewer GPUs")
    return "process", gpus, 0, 0


class Lane:
    """One device's share of the headline: its handles, its `sets` batches, its launch
    stream (the device's current torch stream) and the captured graph of K steps.

    With `streams` > 1 the graph forks: consecutive steps (independent batches) alternate
    between that many streams, one handle each, joined at the end, so a step's input loads
    and factorisation run while the previous step's stores drain instead of after its
    kernel has ended.  Step k uses batch k % sets on stream
    k % streams: concurrent steps never share a batch, and the steps that do share one run
    in order on one stream."""

    def __init__(self, dev: int, gpu_index: int, B: int, M: int, sets: int, method: int, streams: int = 1):
        import torch
        from trajectory_generator_ros2_amd import synthetic as S
        from trajectory_generator_ros2_amd.solver import Solver
        assert streams >= 1 and sets % streams == 0, "sets must be a multiple of streams"
        self.dev, self.B, self.M, self.nstreams = dev, B, M, streams
        with torch.cuda.device(dev):
            self.solvers = [Solver(dev, method) for _ in range(streams)]
            self.solver = self.solvers[0]
            self.bufs = []
            for i in range(sets):
                _, Wi, Ti = S.uniform_batch(B, M, seed=S.SEED + gpu_index + 7919 * i)
                if i == 0:
                    self.W, self.T = Wi, Ti
                self.bufs.append((torch.from_numpy(Wi).to(dev), torch.from_numpy(Ti).to(dev),
                                  torch.empty((B, M, 3, 8), dtype=torch.float64, device=dev),
                                  torch.full((B,), -1, dtype=torch.int32, device=dev)))
            self.stream = torch.cuda.current_stream(dev)
            self.ev0 = torch.cuda.Event(enable_timing=True)
            self.ev1 = torch.cuda.Event(enable_timing=True)
        self.graph = None
        sp = self.stream.cuda_stream
        _solve = self.solver._L.tgms_solve_uniform_device
        self._args = [(self.solver._h, B, M, b[0].data_ptr(), b[1].data_ptr(), None, b[2].data_ptr(),
                       b[3].data_ptr(), ctypes.c_void_p(sp)) for b in self.bufs]
        self._solve = _solve

    def step(self, k: int):
        st = self._solve(*self._args[k % len(self._args)])
        if st != 0:
            raise RuntimeError(f"tgms_solve_uniform_device on device {self.dev}: status {st}: "
                               f"{self.solver.last_error()}")

    def capture(self, K: int, streams: int = 0):
        """The K steps captured once into a HIP graph (thread-local capture: another
        thread -- the RCCL watchdog at N > 1 ranks -- may keep making HIP calls); `streams`
        (default: the lane's) launch streams, forked from and joined to the capture stream."""
        import torch
        n = streams or self.nstreams
        with torch.cuda.device(self.dev):
            cap = torch.cuda.Stream(device=self.dev)
            side = [torch.cuda.Stream(device=self.dev) for _ in range(n - 1)]
            cap.wait_stream(self.stream)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
                for s in side:
                    s.wait_stream(cap)
                for k in range(K):
                    dWk, dTk, dCk, dSk = self.bufs[k % len(self.bufs)]
                    i = k % n
                    st = cap if i == 0 else side[i - 1]
                    self.solvers[i].solve_uniform_device(self.B, self.M, dWk, dTk, dCk, dSk, stream=st.cuda_stream)
                for s in side:
                    cap.wait_stream(s)
            self.stream.wait_stream(cap)
            g.replay()  # warm replay (graph upload)
            torch.cuda.synchronize(self.dev)
        self.graph = g

    def failures(self) -> int:
        return sum(int((b[3] != 0).sum().item()) for b in self.bufs)

    def reset_outputs(self):
        """Every set's coefficients to NaN and statuses to -1 (no solve writes -1), so a
        check after a timed region sees only what that region wrote."""
        import torch
        with torch.cuda.device(self.dev):
            for b in self.bufs:
                b[2].fill_(float("nan"))
                b[3].fill_(-1)
            torch.cuda.synchronize(self.dev)

    def verify(self, K: int) -> dict:
        """After a timed region of K steps: every set a step wrote (set k % sets for k < K)
        has status 0 everywhere and coefficients bit-identical to a fresh one-stream solve
        of the same batch by this lane's first handle (outside any graph)."""
        import torch
        stepped = sorted({k % len(self.bufs) for k in range(K)})
        status_ok, equal = True, True
        with torch.cuda.device(self.dev):
            ref = torch.empty_like(self.bufs[0][2])
            rst = torch.empty_like(self.bufs[0][3])
            for i in stepped:
                dW, dT, dC, dS = self.bufs[i]
                status_ok &= bool((dS == 0).all().item())
                ref.fill_(float("nan"))
                rst.fill_(-1)
                self.solver.solve_uniform_device(self.B, self.M, dW, dT, ref, rst, stream=self.stream.cuda_stream)
                torch.cuda.synchronize(self.dev)
                equal &= bool(torch.equal(ref, dC)) and bool((rst == 0).all().item())
        return {"sets_checked": len(stepped), "sets": len(self.bufs), "status_ok": status_ok,
                "bitwise_equal_one_stream_resolve": equal}


def _timed_multi(fn, dev0_stream, reps: int, devs):
    """Run fn() `reps` times after one warm call; wall clock between synchronisations of
    every device of the process, plus HIP events on device 0's stream."""
    import torch
    fn()
    for d in devs:
        torch.cuda.synchronize(d)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(dev0_stream)
    for _ in range(reps):
        fn()
    e1.record(dev0_stream)
    for d in devs:
        torch.cuda.synchronize(d)
    wall = (time.perf_counter() - t0) / reps * 1e3
    return wall, e0.elapsed_time(e1) / reps


def config4_full_line(devs, ref_solver, reps=3, B_total=1048576, M=10):
    """Config 4 at its stated size through the library's own multi-GPU path: ONE
    tgms_solve_batch_multi_device call over len(devs) devices solves 1,048,576 x M = 10
    (2.0 GB of coefficients) held on device 0: contiguous shards, device 0 scatters the
    other shards' inputs piece by piece over RCCL and gathers their coefficients back
    while the next piece is solved (tgms_capi.hip multi_run).  At one device the shard
    is the whole batch, solved in place.  Check: slices at the start, the end and every
    shard boundary re-solved by a single-device handle, bit for bit."""
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import Solver, plan_shards
    n = len(devs)
    so, W, T = S.uniform_batch(B_total, M)
    with torch.cuda.device(0):
        dso = torch.from_numpy(so).cuda(0)
        dW = torch.from_numpy(W.reshape(-1, 3)).cuda(0)
        dT = torch.from_numpy(T.reshape(-1)).cuda(0)
        dC = torch.empty((B_total * M, 3, 8), dtype=torch.float64, device="cuda:0")
        dS = torch.full((B_total,), -1, dtype=torch.int32, device="cuda:0")
        stream = torch.cuda.current_stream(0)
        mh = Solver(device_count=n)
        try:
            wall, ev = _timed_multi(lambda: mh.solve_batch_multi_device(so, dso, dW, dT, dC, dS,
                                                                        stream=stream.cuda_stream),
                                    stream, reps, devs)
        finally:
            mh.close()
        bad = int((dS != 0).sum().item())
        bounds = [int(b) for b in plan_shards(so, n)]
        chk, k = [], 512
        for b in sorted(set([0, B_total - k] + [max(0, c - k // 2) & ~1 for c in bounds[1:-1]])):
            ref = torch.empty((k * M, 3, 8), dtype=torch.float64, device="cuda:0")
            ref_solver.solve_uniform_device(k, M, dW[b * (M + 1):(b + k) * (M + 1)],
                                            dT[b * M:(b + k) * M], ref, stream=stream.cuda_stream)
            torch.cuda.synchronize(0)
            chk.append(bool(torch.equal(ref, dC[b * M:(b + k) * M])))
    gathered = B_total - (bounds[1] - bounds[0])
    return {"workload": f"config4 (full): {B_total} trajectories x {M} segments in one tgms_solve_batch_multi_device "
                        f"call over {n} device(s), inputs and the 2.0 GB of coefficients on device 0",
            "devices": n, "ms_per_call": wall, "ms_per_call_events_dev0": ev,
            "trajectories_per_s": B_total / (wall * 1e-3),
            "shard_bounds": bounds, "trajectories_gathered_over_rccl": gathered,
            "bytes_gathered": gathered * M * 24 * 8, "status_failures": bad,
            "bit_equal_single_device_slices": all(chk), "slices_checked": len(chk)}


def config5_full_line(devs, reps=3, B_total=1048576, iters=10, k_T=1.0, eta=0.1):
    """Config 5 at its stated size through the library's multi-GPU path: ONE
    tgms_refine_loop_multi_device call over len(devs) devices: 1,048,576 ragged
    trajectories (M ~ U{2..16}), `iters` time-refinement steps + the final solve, the
    shards cost-balanced (tgms_plan_shards), times / costs / coefficients gathered to
    device 0.  The times are reset from a device copy before every call (outside the
    events)."""
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import Solver
    n = len(devs)
    so, W, T = S.ragged_batch(B_total, 2, 16)
    B, Sg = len(so) - 1, int(so[-1])
    with torch.cuda.device(0):
        d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda(0)
        dso, dW, T0 = d(so), d(W), d(T)
        dT = torch.empty_like(T0)
        dC = torch.empty((Sg, 3, 8), dtype=torch.float64, device="cuda:0")
        dcost = torch.empty((B,), dtype=torch.float64, device="cuda:0")
        dst = torch.full((B,), -1, dtype=torch.int32, device="cuda:0")
        stream = torch.cuda.current_stream(0)
        mh = Solver(device_count=n)
        try:
            def run():
                dT.copy_(T0)
                mh.refine_loop_multi_device(so, dso, dW, dT, k_T, eta, iters, dC, dcost, dst,
                                            stream=stream.cuda_stream)
            wall, _ = _timed_multi(run, stream, reps, devs)
            # events around the call alone; the host time of the call (offsets scan, shard
            # plan, graph replays, RCCL groups) with every device idle
            run()
            torch.cuda.synchronize(0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            evs, host = [], []
            for _ in range(reps):
                dT.copy_(T0)
                for dd in devs:
                    torch.cuda.synchronize(dd)
                e0.record(stream)
                h0 = time.perf_counter()
                mh.refine_loop_multi_device(so, dso, dW, dT, k_T, eta, iters, dC, dcost, dst,
                                            stream=stream.cuda_stream)
                host.append((time.perf_counter() - h0) * 1e3)
                e1.record(stream)
                torch.cuda.synchronize(0)
                evs.append(e0.elapsed_time(e1))
        finally:
            mh.close()
        bad = int((dst != 0).sum().item())
        finite = bool(torch.isfinite(dcost).all().item())
    ms = sorted(evs)[len(evs) // 2]
    return {"workload": f"config5 (full): {B_total} ragged trajectories (M~U{{2..16}}, {Sg} segments), {iters} "
                        f"refinement steps + final solve in one tgms_refine_loop_multi_device call over {n} "
                        f"device(s)",
            "devices": n, "ms_per_call": ms, "ms_per_call_wall_incl_time_reset": wall,
            "host_ms_per_call": sorted(host)[len(host) // 2],
            "trajectories_per_s": B / (ms * 1e-3), "segments": Sg, "k_T": k_T, "eta": eta,
            "status_failures": bad, "costs_finite": finite}


def full_lines_child(n: int, timeout_s: float) -> dict:
    """config4_full / config5_full over devices 0..n-1, run by `bench.py --gpus n
    --full-lines-only` as a child process (started fresh, not forked from this GPU
    process's state) under `timeout_s`; its JSON, or an error record."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(n), "--full-lines-only", "--cpu-seconds", "0"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"the {n}-device library side lines exceeded {timeout_s:.0f} s and were abandoned"}
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"child exited {r.returncode}: {r.stderr.strip()[-400:]}"}
    return json.loads(lines[-1])


def _side(name, fn):
    """A side line that fails reports its error instead of ending the run."""
    try:
        return fn()
    except Exception as exc:  # noqa: BLE001 -- recorded in the JSON line
        print(f"bench: side line {name} failed: {type(exc).__name__}: {exc}", file=sys.stderr)
        return {"error": f"{type(exc).__name__}: {exc}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of the run.  Under torch.distributed.run: one rank per GPU (WORLD_SIZE must equal "
                         "it).  Without a launcher: one process drives devices 0..N-1 (one handle and stream "
                         "per device for the headline; the library's multi-GPU handle for the config-4/5 lines)")
    ap.add_argument("--backend", default="nccl",
                    help="process-group backend at N > 1 ranks (nccl = RCCL; gloo only to rehearse the N > 1 "
                         "control flow with several ranks on one GPU)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="trajectories per GPU")
    ap.add_argument("--segments", type=int, default=10)
    ap.add_argument("--sets", type=int, default=4,
                    help="independent batches the timed steps rotate over (a fresh batch every step)")
    ap.add_argument("--method", choices=["reduced", "dense"], default="reduced")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: the K timed steps replayed from one captured HIP graph; 0: K Python-level launches")
    ap.add_argument("--streams", type=int, default=4,
                    help="launch streams per device in the captured graph: consecutive steps (independent "
                         "batches) alternate between them, one handle each, so a step's loads and "
                         "factorisation overlap the previous step's store drain; 1: steps back to back. The "
                         "roofline is timed separately with one stream (kernel durations, as rocprofv3 sees them)")
    ap.add_argument("--dense-steps", type=int, default=1,
                    help="steps of the dense-KKT side line (0: skip).  The dense KKT is a cross-check method "
                         "(DESIGN.md section 4): one timing")
    ap.add_argument("--band-steps", type=int, default=5, help="steps of the band-KKT side line (0: skip)")
    ap.add_argument("--config2", type=int, default=1,
                    help="config-2 side line (1,024 x M = 3: every method's latency, host path, CPU oracle): 1/0")
    ap.add_argument("--sample-traj", type=int, default=4096,
                    help="trajectories of the sampler side line at dt = 0.01 (0: skip)")
    ap.add_argument("--config5", type=int, default=1,
                    help="config-5 side lines (ragged + refinement: one GPU's share, and the full batch): 1/0")
    ap.add_argument("--cache-resident", type=int, default=1,
                    help="side line: the same batch every launch (its 148.6 MB stay in the Infinity Cache): 1/0")
    ap.add_argument("--config4", type=int, default=1,
                    help="config-4 side lines (131,072/GPU shard; the full 1,048,576 batch through the "
                         "library's multi-GPU call, or a per-rank RCCL gather under a launcher): 1/0")
    ap.add_argument("--node-line", type=int, default=1, help="config-1 node-path latency side line: 1/0")
    ap.add_argument("--host-line", type=int, default=1, help="PCIe-inclusive host-buffer side line: 1/0")
    ap.add_argument("--uniform-large-m", type=int, default=1,
                    help="uniform M = 12/14/16 side line (fresh batches): 1/0")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="0: skip the CPU baseline")
    ap.add_argument("--full-lines-only", action="store_true",
                    help="internal: print only the config4_full / config5_full lines over devices 0..N-1 (the "
                         "parent runs them in this child process at N > 1, under a time limit)")
    ap.add_argument("--full-lines-timeout", type=float, default=300.0,
                    help="seconds the N > 1 library multi-GPU side lines may take before they are abandoned")
    args = ap.parse_args()
    # concurrent steps must never share a batch: step k runs batch k % sets on stream k % streams
    if args.graph and args.streams > 1 and max(1, args.sets) % args.streams:
        raise SystemExit(f"bench.py: --sets {args.sets} must be a multiple of --streams {args.streams}")

    import torch
    import torch.distributed as dist

    mode, n_total, rank, local = resolve_topology(args.gpus, os.environ, torch.cuda.device_count())
    world = n_total if mode == "ranks" else 1          # processes
    if mode == "ranks" and world > 1:
        local = local % max(torch.cuda.device_count(), 1) if args.backend == "gloo" else local
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
        devs = [local]
    elif mode == "ranks":
        devs = [0]
    else:
        devs = list(range(n_total))
    torch.cuda.set_device(devs[0])

    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_DENSE_KKT, METHOD_REDUCED

    if args.full_lines_only:
        from trajectory_generator_ros2_amd.solver import Solver
        with Solver(devs[0]) as ref:
            out = {"config4_full": _side("config4_full", lambda: config4_full_line(devs, ref)),
                   "config5_full": _side("config5_full", lambda: config5_full_line(devs))}
        print(json.dumps(out), flush=True)
        return

    B, M, sets = args.batch, args.segments, max(1, args.sets)
    method = METHOD_DENSE_KKT if args.method == "dense" else METHOD_REDUCED
    # this process's devices, each with its own shard of the job: `sets` independent
    # batches of independent trajectories (set 0: seed + GPU index, as every side line uses)
    nstreams = max(1, args.streams) if args.graph else 1
    lanes = [Lane(d, rank if mode == "ranks" else d, B, M, sets, method, nstreams) for d in devs]
    torch.cuda.set_device(devs[0])
    lane0 = lanes[0]
    solver, dev, stream = lane0.solver, lane0.dev, lane0.stream
    W, T = lane0.W, lane0.T
    dW, dT, dC, dS = lane0.bufs[0]
    sp = stream.cuda_stream

    def barrier():
        if world > 1:
            dist.barrier()

    def sync_all():
        for L in lanes:
            torch.cuda.synchronize(L.dev)

    def all_ranks(x: float, op):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    for L in lanes:
        for k in range(max(args.warmup, sets)):
            L.step(k)
        for sv in L.solvers[1:]:  # the other streams' handles: first calls outside any capture
            b = L.bufs[0]
            sv.solve_uniform_device(B, M, b[0], b[1], b[2], b[3], stream=L.stream.cuda_stream)
    sync_all()
    assert all(L.failures() == 0 for L in lanes), "solver reported failures"

    K = args.steps
    # The K steps are captured once into a HIP graph per device (torch.cuda.CUDAGraph over
    # the library's launches) and replayed as one submission, so a slow or busy host
    # cannot starve the GPU between ~30 us launches; every step is still one full solve
    # of a batch.  HIP events on each device's launch stream bracket its timed region;
    # the average launch duration is their elapsed time / K.  --graph 0: K Python-level
    # launches.  Every rank times the same launch mode: if capture fails anywhere, all
    # fall back.
    capture_error = None
    if args.graph:
        try:
            for L in lanes:
                L.capture(K)
        except Exception as exc:  # capture unsupported here: time the Python loop instead
            capture_error = f"{type(exc).__name__}: {exc}"
            print(f"bench: HIP graph capture failed ({capture_error}); timing the launch loop", file=sys.stderr)
            for L in lanes:
                L.graph = None
            sync_all()
        ok = 1.0 if all(L.graph is not None for L in lanes) else 0.0
        if all_ranks(ok, dist.ReduceOp.MIN if world > 1 else None) < 1.0:
            for L in lanes:
                L.graph = None  # some rank could not capture: every rank times the launch loop
    graphed = all(L.graph is not None for L in lanes)
    # the timed region must prove its own output: every set back to NaN / status -1 first
    for L in lanes:
        L.reset_outputs()
    barrier()
    sync_all()
    t0 = time.perf_counter()
    for L in lanes:  # every device's K steps issued from this one thread, then all run
        L.ev0.record(L.stream)
        if graphed:
            with torch.cuda.device(L.dev):
                L.graph.replay()
        else:
            for k in range(K):
                L.step(k)
        L.ev1.record(L.stream)
    sync_all()
    barrier()
    el = all_ranks(time.perf_counter() - t0, dist.ReduceOp.MAX if world > 1 else None)
    launch_each = [L.ev0.elapsed_time(L.ev1) / K for L in lanes]
    step_ms_max = all_ranks(max(launch_each), dist.ReduceOp.MAX if world > 1 else None)
    # outside the timed region: what the K steps wrote, against a one-stream re-solve
    checks = [L.verify(K) for L in lanes]
    ver_ok = all(c["status_ok"] and c["bitwise_equal_one_stream_resolve"] for c in checks)
    ver_ok = all_ranks(1.0 if ver_ok else 0.0, dist.ReduceOp.MIN if world > 1 else None) == 1.0
    assert ver_ok, f"the timed region's output failed verification: {checks}"
    timed_set0 = lane0.bufs[0][2][: min(B, 65536)].cpu().numpy().reshape(-1, 3, 8) if rank == 0 else None
    launch_mode = ("hip_graph_of_K_steps" + (f"_over_{nstreams}_streams" if nstreams > 1 else "")) if graphed \
        else "python_loop"
    for L in lanes:
        L.graph = None
    # The roofline is the kernel's own rate: with steps overlapping across streams a step's
    # share of the timed region is shorter than a kernel's duration, so the K steps are
    # timed again back to back on one stream (the same kernels rocprofv3 reports, their
    # durations adding up to the region).
    if graphed and nstreams > 1:
        for L in lanes:
            L.capture(K, streams=1)
        barrier()
        sync_all()
        for L in lanes:
            L.ev0.record(L.stream)
            with torch.cuda.device(L.dev):
                L.graph.replay()
            L.ev1.record(L.stream)
        sync_all()
        barrier()
        kernel_each = [L.ev0.elapsed_time(L.ev1) / K for L in lanes]
        assert all(L.failures() == 0 for L in lanes), "solver reported failures"
        for L in lanes:
            L.graph = None
    else:
        kernel_each = launch_each
    launch_ms_max = all_ranks(max(kernel_each), dist.ReduceOp.MAX if world > 1 else None)
    launch_ms_min = all_ranks(min(kernel_each), dist.ReduceOp.MIN if world > 1 else None)

    per_launch = launch_stats(solver, B, M, lane0.bufs, stream)
    cache_res = None
    if args.cache_resident and args.method == "reduced":
        cache_res = cache_resident_line(solver, B, M, lane0.bufs[0], stream)
    # the side lines use device 0's set 0 only
    for L in lanes:
        L.bufs = L.bufs[:1]
        L._args = L._args[:1]
    torch.cuda.empty_cache()

    # dense-KKT side line (the survey's literal formulation), same inputs, same GPU
    dense = None
    if args.dense_steps > 0 and args.method == "reduced" and M <= 10:
        solver.set_method(METHOD_DENSE_KKT)
        dC2 = torch.empty_like(dC)
        solver.solve_uniform_device(B, M, dW, dT, dC2, dS, stream=sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.dense_steps):
            solver.solve_uniform_device(B, M, dW, dT, dC2, dS, stream=sp)
        e1.record(stream)
        torch.cuda.synchronize()
        dms = e0.elapsed_time(e1) / args.dense_steps
        diff = (dC2 - dC).abs().amax(dim=(1, 3)) / dC.abs().amax(dim=(1, 3)).clamp_min(1e-300)
        gfl = dense_flops_per_traj(M) * B / (dms * 1e-3) / 1e12
        dense = {"value": B / (dms * 1e-3), "ms_per_step": dms,
                 "fp64_tflops_algorithmic": gfl, "fp64_peak_tflops": FP64_PEAK_TFS,
                 "max_rel_diff_vs_reduced": float(diff.max().item())}
        solver.set_method(method)
        del dC2

    # band-KKT side line: the same literal KKT and partial-pivoting LU in the order in
    # which it is banded (tgms_band.hip), same inputs, same GPU
    band = None
    if args.band_steps > 0 and args.method == "reduced":
        solver.set_method(METHOD_BAND_KKT)
        dC3 = torch.empty_like(dC)
        solver.solve_uniform_device(B, M, dW, dT, dC3, dS, stream=sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.band_steps):
            solver.solve_uniform_device(B, M, dW, dT, dC3, dS, stream=sp)
        e1.record(stream)
        torch.cuda.synchronize()
        assert int((dS != 0).sum().item()) == 0, "band KKT reported failures"
        bms = e0.elapsed_time(e1) / args.band_steps
        diff = (dC3 - dC).abs().amax(dim=(1, 3)) / dC.abs().amax(dim=(1, 3)).clamp_min(1e-300)
        band = {"value": B / (bms * 1e-3), "ms_per_step": bms,
                "fp64_tflops_algorithmic": band_flops_per_traj(M) * B / (bms * 1e-3) / 1e12,
                "flops_per_traj": band_flops_per_traj(M), "fp64_peak_tflops": FP64_PEAK_TFS,
                "max_rel_diff_vs_reduced": float(diff.max().item())}
        solver.set_method(METHOD_REDUCED)
        del dC3

    # N > 1 (or TGMS_BENCH_FULL_CHILD=1, to rehearse it on one GPU): the full-size lines
    # run in a child process
    child_full = len(devs) > 1 or os.environ.get("TGMS_BENCH_FULL_CHILD") == "1"
    config5 = config5_full = None
    if args.config5 and M == 10:
        config5 = config5_line(solver, dev, stream, world, rank)
        if world == 1 and len(devs) == 1 and not child_full:
            config5_full = _side("config5_full", lambda: config5_full_line(devs))

    config4 = config4_full = None
    if args.config4 and M == 10:
        config4 = config4_line(solver, M, dev, stream, world, rank)
        if world == 1 and len(devs) == 1 and not child_full:
            config4_full = _side("config4_full", lambda: config4_full_line(devs, solver))

    if world == 1 and child_full and (args.config4 or args.config5) and M == 10:
        # the library's own multi-GPU path (one RCCL communicator per device inside this
        # process's library handle) runs in a child process under a time limit: a stuck
        # collective then costs this side line, never the headline
        full = full_lines_child(len(devs), args.full_lines_timeout)
        if args.config4:
            config4_full = full.get("config4_full", full)
        if args.config5:
            config5_full = full.get("config5_full", full)

    config2 = None
    if args.config2 and args.method == "reduced" and rank == 0:
        config2 = _side("config2", lambda: config2_line(solver, dev, stream))
        solver.set_method(METHOD_REDUCED)

    sampler = None
    if args.sample_traj > 0:
        sampler = sampler_line(solver, args.sample_traj, M, W, T, dC, dev, stream)

    uniform_m = None
    if args.uniform_large_m and args.method == "reduced":
        uniform_m = _side("uniform_large_m", lambda: uniform_large_m_line(solver, dev, stream))

    host = None
    if args.host_line and rank == 0:
        host = host_line(solver, B, M, W, T)

    node = node_host = None
    if args.node_line and rank == 0:
        node = node_line()
        node_host = _side("node_config1_host_backend", host_backend_node_line)

    # rank-0-only host work, after every GPU timing (the other ranks wait at the
    # final barrier)
    cpu = None
    oracle_check = {"skipped": "--cpu-seconds 0 (the check is the CPU baseline's own output)"}
    if rank == 0 and args.cpu_seconds > 0:
        cpu, oracle_check = cpu_baseline(B, M, args.cpu_seconds, check=timed_set0)

    if rank == 0:
        bpl = algorithmic_bytes_per_traj(M) * B
        achieved = bpl / (launch_ms_max * 1e-3) / 1e9
        key = f"B{B}_M{M}_{args.method}_sets{sets}"
        traffic = load_traffic(key)
        value = n_total * B * K / el
        if mode == "ranks":
            parallelism = f"shard{n_total}: one rank per GPU (independent trajectories, no collective)"
        else:
            parallelism = (f"shard{n_total}: one process, one handle + stream + graph per device, launched from one "
                           f"thread (independent trajectories, no collective)")
        line = {
            "metric": "min-snap trajectories/sec (10-seg, order-7, 3-axis) at batch=65k; 1/2/4/8 GPU",
            "value": value,
            "unit": "trajectories/s",
            "n_gpus": n_total,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": el / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md 8(d): seed 20251015+GPU index(+7919 i for batch i), room-bound uniform "
                    "waypoints, T=clip(|dw|/1m/s,0.5,10), rest-to-rest)",
            "config": {"workload": f"config3: {B} trajectories/GPU x {M} segments, order 7, 3 axes, "
                                   f"coefficients [traj][seg][axis][8] fp64 in HBM; a fresh batch every step "
                                   f"({sets} batches rotated, {sets * bpl / 1e6:.0f} MB per GPU), "
                                   f"{nstreams} launch stream(s) per device",
                       "batch_per_gpu": B, "segments": M, "sets": sets, "method": args.method,
                       "launch": launch_mode, "streams_per_device": nstreams,
                       "processes": world, "devices_per_process": len(devs),
                       "parallelism": parallelism},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_source": (f"{TRAFFIC_FILE}[{key}]: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                                            f"passes of this command (scripts/gpu_profile.sh), not this run")
                         if traffic is not None else None,
                         "kernel": (f"k_dense_kkt<{M}>" if args.method == "dense" else
                                    f"k_lane_uniform<{M}>" if M % 2 == 0 else f"k_reduced_uniform<{M}>"),
                         "launch_ms": launch_ms_max,
                         # the measured floor of this byte mix with NO compute (read the inputs,
                         # write the coefficients, fresh buffers, best occupancy and rounds:
                         # scripts/micro/occstore.hip, profiles/archive/r03_runstore_occ.txt): the
                         # fraction of the attainable rate the kernel reaches
                         "floor_us": BYTE_MIX_FLOOR_US if (B, M) == (65536, 10) else None,
                         "floor_frac": (BYTE_MIX_FLOOR_US / (launch_ms_max * 1e3)) if (B, M) == (65536, 10) else None,
                         "floor_source": "profiles/archive/r03_runstore_occ.txt (reads + stores, no compute, 2 waves/SIMD, "
                                         "4 rounds: 28.6 us for 22.5 MB read + 126 MB written)",
                         "launch_ms_rank_min": launch_ms_min, "launch_ms_rank_max": launch_ms_max,
                         "launch_ms_how": ("the K steps back to back on one stream, timed after the headline "
                                           "region (kernel durations)" if nstreams > 1 and graphed else
                                           "the headline region's events / K"),
                         "algorithmic_bytes_per_launch": bpl,
                         # the headline region itself: steps overlapping across the streams
                         "pipelined": {"streams": nstreams, "ms_per_step_events": step_ms_max,
                                       "achieved": bpl / (step_ms_max * 1e-3) / 1e9,
                                       "frac": bpl / (step_ms_max * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                       "floor_us": PIPELINED_FLOOR_US if (B, M) == (65536, 10) and nstreams > 1
                                       else None,
                                       "floor_frac": (PIPELINED_FLOOR_US / (step_ms_max * 1e3))
                                       if (B, M) == (65536, 10) and nstreams > 1 else None,
                                       "floor_source": "profiles/r06_floor.jsonl (scripts/micro/floor.hip: the same "
                                                       "bytes, no compute, 4 streams in one graph, best occupancy)"}},
            # the timed region's own output: every set reset to NaN /
            # status -1 before it, then bit-compared with a one-stream re-solve and (set 0,
            # rank 0) with the CPU baseline's oracle output
            "verified": bool(ver_ok and (oracle_check.get("ok", True))),
            "verification": {"per_device": checks, "oracle": oracle_check},
            # the same K steps back to back on one stream (rounds 1-4's headline form)
            "value_one_stream": n_total * B / (launch_ms_max * 1e-3),
            "cpu_baseline": cpu,
            "per_launch": per_launch,
            "cache_resident": cache_res,
            "dense_kkt": dense,
            "band_kkt": band,
            "config2": config2,
            "sampler": sampler,
            "config4": config4,
            "config4_full": config4_full,
            "config5": config5,
            "config5_full": config5_full,
            "uniform_large_m": uniform_m,
            "host_path": host,
            "node_config1": node,
            "node_config1_host_backend": node_host,
        }
        if capture_error is not None:
            line["config"]["graph_capture_error"] = capture_error
        print(json.dumps(line), flush=True)
    barrier()
    for L in lanes:
        for sv in L.solvers:
            sv.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
