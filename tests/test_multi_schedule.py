"""CPU: the multi-GPU schedule (tgms_multi_schedule, include/tgms.h) that
tgms_solve_batch_multi_device / tgms_refine_loop_multi_device execute over RCCL, checked
at 2..8 devices without a GPU.

The schedule comes from the host-only planner (csrc/tgms_plan.cpp) that multi_enqueue
consumes verbatim, so what is asserted here is what the HIP/RCCL code issues:
  - shard bounds equal tgms_plan_shards / shard.ragged_bounds;
  - the pieces tile every shard, in order; device 0's shard has no pieces unless
    self-gather is on (it is solved in place);
  - every piece's workspace regions are 256-B aligned, inside the workspace and pairwise
    disjoint (plan block included);
  - every transfer is one send + one recv between device 0 and the piece's device, with
    the piece's own counts and offsets; scatter groups 0..3 hold piece k's inputs of every
    device, gather groups 4..7 its results;
  - executing the schedule on byte buffers (scatter, a stand-in per-piece solve, gather)
    reproduces the stand-in solve of the whole batch exactly, and covers every output
    element exactly once.
"""
import numpy as np
import pytest

from trajectory_generator_ros2_amd import _lib

S = _lib
ALIGN = 256


@pytest.fixture(scope="module")
def lib():
    import os
    from trajectory_generator_ros2_amd.build import LIB_TGMS, build_tgms
    if not os.path.exists(LIB_TGMS):
        build_tgms()
    return _lib.load()


def _batches():
    from trajectory_generator_ros2_amd import synthetic as SY
    return {
        "uniform10": SY.uniform_batch(4096, 10)[0],
        "uniform3_odd": SY.uniform_batch(1001, 3)[0],
        "ragged": SY.ragged_batch(5000, 2, 16, seed=5)[0],
        "tiny": SY.uniform_batch(5, 2)[0],  # fewer trajectories than devices x pieces
    }


SOLVE = S.SCHED_COEFFS | S.SCHED_STATUS
REFINE = S.SCHED_REFINE | S.SCHED_COEFFS | S.SCHED_STATUS | S.SCHED_COST
FLAGS = [SOLVE, SOLVE | S.SCHED_END_DERIVS, SOLVE | S.SCHED_SELF_GATHER, REFINE, REFINE | S.SCHED_END_DERIVS,
         S.SCHED_STATUS]


def _region_sizes(p, flags, ragged, method=0):
    """Bytes of ws_off[0..10]: offsets, permutation (ragged only), W, T, T2, ED, C, status,
    cost, and for a device-planned piece the device grouping's block counts and plan (round 5:
    every refinement batch, uniform ones too, is grouped on the device, laid out as a ragged
    one; round 6: so is a ragged solve with the reduced method, method 0)."""
    n, Sg = p["hi"] - p["lo"], p["s1"] - p["s0"]
    refine = bool(flags & S.SCHED_REFINE)
    dev = refine or (ragged and method == 0)
    ragged = ragged or refine
    return [4 * (n + 1) if ragged else 0, 4 * n if ragged else 0, 8 * 3 * (Sg + n), 8 * Sg, 8 * Sg if refine else 0,
            8 * 18 * n if flags & S.SCHED_END_DERIVS else 0, 8 * 24 * Sg if flags & S.SCHED_COEFFS else 0,
            4 * n, 8 * n if refine else 0, 17 * 4 * ((n + 1023) // 1024) if dev else 0, 1024 if dev else 0]


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("flags", FLAGS)
def test_schedule_structure(lib, n, flags):
    from trajectory_generator_ros2_amd.solver import multi_schedule, plan_shards
    for name, so in _batches().items():
        so = so.astype(np.int64)
        ragged = len(set(np.diff(so).tolist())) > 1
        bounds, ws, P, X = multi_schedule(so, n, 0, flags)
        np.testing.assert_array_equal(bounds, plan_shards(so, n, 0))
        self_gather = bool(flags & S.SCHED_SELF_GATHER)
        # pieces tile every shard, in order
        for d in range(n):
            mine = [p for p in P if p["dev"] == d]
            lo, hi = int(bounds[d]), int(bounds[d + 1])
            if (d == 0 and not self_gather) or hi <= lo:
                assert not mine, (name, d)
                continue
            assert [p["piece"] for p in mine] == list(range(len(mine)))
            assert 1 <= len(mine) <= 4
            assert mine[0]["lo"] == lo and mine[-1]["hi"] == hi
            for a, b in zip(mine, mine[1:]):
                assert a["hi"] == b["lo"]
            for p in mine:
                assert p["lo"] < p["hi"] and p["s0"] == so[p["lo"]] and p["s1"] == so[p["hi"]]
            # workspace regions: aligned, inside, disjoint
            regs = []
            for p in mine:
                for off, size in zip(p["ws_off"], _region_sizes(p, flags, ragged)):
                    assert off % ALIGN == 0
                    if size:
                        assert off + size <= ws[d], (name, d)
                        regs.append((off, off + size))
            regs.sort()
            for (a0, a1), (b0, b1) in zip(regs, regs[1:]):
                assert a1 <= b0, (name, d, regs)
        # transfers: per piece, the piece's own ranges
        by = {(p["dev"], p["piece"]): p for p in P}
        groups = [x["group"] for x in X]
        assert groups == sorted(groups)
        for x in X:
            p = by[(x["dev"], x["piece"])]
            assert 0 <= x["dev"] < n and (x["dev"] > 0 or self_gather)
            assert x["group"] == x["piece"] + (4 if x["gather"] else 0)
            npc, Sg = p["hi"] - p["lo"], p["s1"] - p["s0"]
            exp = {  # array -> (gather?, batch element offset, count, bytes, ws offset index)
                0: (0, (p["s0"] + p["lo"]) * 3, (Sg + npc) * 3, 8, 2),
                1: (x["gather"], p["s0"], Sg, 8, 3),
                2: (0, p["lo"] * 18, npc * 18, 8, 5),
                3: (1, p["s0"] * 24, Sg * 24, 8, 6),
                4: (1, p["lo"], npc, 4, 7),
                5: (1, p["lo"], npc, 8, 8),
                6: (0, p["lo"], npc + 1, 4, 0),
            }[x["array"]]
            assert (x["gather"], x["batch_elem"], x["count"], x["elem_bytes"], x["ws_byte"]) == \
                (exp[0], exp[1], exp[2], exp[3], p["ws_off"][exp[4]]), (name, x)
        # which arrays move: exactly the flags'
        for p in P:
            arrs = sorted((x["gather"], x["array"]) for x in X if (x["dev"], x["piece"]) == (p["dev"], p["piece"]))
            want = [(0, 0), (0, 1)] + ([(0, 2)] if flags & S.SCHED_END_DERIVS else [])
            want += [(1, 3)] if flags & S.SCHED_COEFFS else []
            want += [(1, 4)] if flags & S.SCHED_STATUS else []
            if flags & S.SCHED_REFINE:
                want += [(1, 1), (1, 5)] if flags & S.SCHED_COST else [(1, 1)]
                want += [(0, 6)]  # the offsets slice, planned on the device (uniform batches too)
            elif ragged:
                want += [(0, 6)]  # round 6: a ragged reduced solve is planned on the device too
            assert arrs == sorted(want), (name, arrs)


def _fake_solve(so, W, T):
    """A stand-in per-trajectory 'solve' that depends on every input row the real one reads
    (W rows so[b]+b .. so[b+1]+b, T[so[b]..so[b+1]]) and on the trajectory's local layout."""
    B = so.shape[0] - 1
    C = np.zeros((so[-1], 3, 8))
    st = np.zeros(B, np.int32)
    for b in range(B):
        m = so[b + 1] - so[b]
        for i in range(m):
            s = so[b] + i
            C[s] = (T[s] + W[so[b] + b + i][:, None] * np.arange(1, 9) + W[so[b] + b + i + 1][:, None])
        st[b] = m
    return C, st


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("self_gather", [False, True])
def test_schedule_executes_to_the_whole_batch_result(lib, n, self_gather):
    """Run the schedule on byte buffers: scatter from the device-0 arrays into per-device
    workspaces, the stand-in solve of every piece from its workspace, gather back; device
    0's shard (when not self-gathered) is solved in place.  The result equals the stand-in
    solve of the whole batch, and every output element is written exactly once."""
    from trajectory_generator_ros2_amd import synthetic as SY
    from trajectory_generator_ros2_amd.solver import multi_schedule
    so, W, T = SY.ragged_batch(3000, 1, 16, seed=n)
    so = so.astype(np.int64)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    flags = SOLVE | (S.SCHED_SELF_GATHER if self_gather else 0)
    bounds, ws, P, X = multi_schedule(so, n, 0, flags)
    Cref, stref = _fake_solve(so, W, T)
    batch = {0: W.copy().view(np.uint8).reshape(-1), 1: T.copy().view(np.uint8).reshape(-1),
             3: np.zeros(Cref.size * 8, np.uint8), 4: np.zeros(stref.size * 4, np.uint8),
             6: so.astype(np.int32).view(np.uint8).reshape(-1)}
    written = {3: np.zeros(Cref.size, np.int32), 4: np.zeros(stref.size, np.int32)}
    wsb = [np.zeros(int(w), np.uint8) for w in ws]
    for x in [x for x in X if not x["gather"]]:
        nb = x["count"] * x["elem_bytes"]
        src = batch[x["array"]][x["batch_elem"] * x["elem_bytes"]:][:nb]
        assert src.size == nb
        wsb[x["dev"]][x["ws_byte"]:x["ws_byte"] + nb] = src
    for p in P:
        w = wsb[p["dev"]]
        npc, Sg = p["hi"] - p["lo"], p["s1"] - p["s0"]
        so_l = so[p["lo"]:p["hi"] + 1] - so[p["lo"]]
        # the raw offsets slice the device plans from arrived with the inputs (round 6)
        raw = w[p["ws_off"][0]:][:4 * (npc + 1)].view(np.int32)
        np.testing.assert_array_equal(raw - raw[0], so_l)
        Wl = w[p["ws_off"][2]:][:8 * 3 * (Sg + npc)].view(np.float64).reshape(-1, 3)
        Tl = w[p["ws_off"][3]:][:8 * Sg].view(np.float64)
        Cl, stl = _fake_solve(so_l, Wl, Tl)
        w[p["ws_off"][6]:p["ws_off"][6] + Cl.nbytes] = Cl.view(np.uint8).reshape(-1)
        w[p["ws_off"][7]:p["ws_off"][7] + stl.nbytes] = stl.view(np.uint8)
    for x in [x for x in X if x["gather"]]:
        nb = x["count"] * x["elem_bytes"]
        dst = batch[x["array"]]
        dst[x["batch_elem"] * x["elem_bytes"]:][:nb] = wsb[x["dev"]][x["ws_byte"]:x["ws_byte"] + nb]
        written[x["array"]][x["batch_elem"]:x["batch_elem"] + x["count"]] += 1
    if not self_gather:  # device 0's shard in place
        b1 = int(bounds[1])
        C0, st0 = _fake_solve(so[:b1 + 1], W, T)
        batch[3][:C0.nbytes] = C0.view(np.uint8).reshape(-1)
        batch[4][:st0.nbytes] = st0.view(np.uint8)
        written[3][:C0.size] += 1
        written[4][:b1] += 1
    assert (written[3] == 1).all() and (written[4] == 1).all()
    np.testing.assert_array_equal(batch[3].view(np.float64).reshape(Cref.shape), Cref)
    np.testing.assert_array_equal(batch[4].view(np.int32), stref)


def test_schedule_arguments(lib):
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, TgmsError
    from trajectory_generator_ros2_amd.solver import multi_schedule
    b, ws, P, X = multi_schedule(np.zeros(1, np.int32), 4, 0, SOLVE)
    assert list(b) == [0] * 5 and not P and not X
    for so, n in [(np.array([0, 2, 2], np.int32), 2), (np.array([0, 17], np.int32), 2),
                  (np.array([0, 3], np.int32), 0)]:
        with pytest.raises(TgmsError) as e:
            multi_schedule(so, n, 0, SOLVE)
        assert e.value.status == ERR_INVALID_ARG


def test_refine_schedule_leaves_per_trajectory_checks_to_the_devices(lib):
    """Round 5: the refinement loop's host work reads only the cuts.  A bad M strictly
    inside a piece passes the host (its device's k_plan_scatter rejects that piece:
    tests/test_gpu_multi.py::test_refine_multi_bad_offsets_fail_on_the_device); offsets
    whose shard or piece spans no M in 1..16 can give (the workspaces are sized from them) are
    refused; a decrease that the cuts do not expose is again the devices' to reject."""
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, TgmsError
    from trajectory_generator_ros2_amd import synthetic as SY
    from trajectory_generator_ros2_amd.solver import multi_schedule
    so = SY.ragged_batch(4000, 2, 16, seed=9)[0].astype(np.int32)
    bad = so.copy()
    bad[1001:] += 20  # trajectory 1000 gets M + 20
    with pytest.raises(TgmsError):
        multi_schedule(bad, 4, 2, SOLVE)  # band method: host-planned pieces, validated on the host
    for flags in (REFINE, SOLVE):  # round 6: a reduced ragged solve leaves it to the devices too
        b, _, P, _ = multi_schedule(bad, 4, 0, flags)
        assert not any(p["lo"] == 1000 or p["hi"] == 1001 for p in P)  # strictly inside a piece
    for so_dec in ([0, 2, 4, 6, 3, 10, 12, 14, 16], [0, 2, 4, 1, 8, 10, 12, 14, 16]):
        b, _, P, _ = multi_schedule(np.array(so_dec, np.int32), 4, 0, REFINE)
        for q in P:
            assert q["hi"] - q["lo"] <= q["s1"] - q["s0"] <= 16 * (q["hi"] - q["lo"])
    for so_bad in ([0, 3, 100], [0, 3, 3], [0, 2, 4, 6, 8, 10, 12, 14, 9]):
        with pytest.raises(TgmsError) as e:
            multi_schedule(np.array(so_bad, np.int32), 4, 0, REFINE)
        assert e.value.status == ERR_INVALID_ARG


def test_shard_cuts_by_binary_search_match_the_prefix_sum_rule():
    """Round 5: the reduced / band planner cuts ragged batches by binary search over the
    integer running cost 2 (b + 1) + so[b + 1] (no pass over the batch), and the pieces of a
    shard from the shard's own offsets slice; both must give shard.ragged_bounds' cuts."""
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as SY
    from trajectory_generator_ros2_amd.solver import multi_schedule, plan_shards
    for seed, (B, lo, hi) in enumerate([(1, 1, 16), (7, 2, 16), (5000, 2, 16), (4096, 1, 3), (333, 15, 16)]):
        so = SY.ragged_batch(B, lo, hi, seed=seed)[0].astype(np.int64)
        for parts in (1, 2, 3, 4, 8, 13):
            np.testing.assert_array_equal(plan_shards(so, parts, 0), SH.ragged_bounds(so, parts))
        _, _, P, _ = multi_schedule(so, 8, 0, REFINE)
        for d in range(1, 8):  # a shard's pieces: the same rule applied to the shard's slice
            mine = [p for p in P if p["dev"] == d]
            if not mine:
                continue
            a, b = mine[0]["lo"], mine[-1]["hi"]
            want = sorted(set(int(x) for x in SH.ragged_bounds(so[a:b + 1] - so[a], 4)))
            assert [p["lo"] - a for p in mine] + [b - a] == want


def test_schedule_host_time_at_8_devices(lib):
    """Round 5: the host-side work of a multi-GPU refinement call
    before its first RCCL transfer -- the offsets' ends and cuts, the whole schedule (shards
    and pieces by binary search, workspaces, transfers) -- for 1,048,576 ragged trajectories
    over 8 devices, timed on the C call alone (tgms_multi_schedule with TGMS_SCHED_REFINE
    runs exactly that work): median <= 0.1 ms.  Round 6: the reduced
    solve's schedule as well (its pieces are grouped on the devices; round 5 kept a
    validation pass, 0.71 ms); the band method's, which keeps it, and a uniform batch's
    detection pass are printed beside."""
    import ctypes
    import time
    from trajectory_generator_ros2_amd import _lib
    from trajectory_generator_ros2_amd import synthetic as SY
    so = SY.ragged_batch(1 << 20, 2, 16, seed=3)[0].astype(np.int32)
    B, n = len(so) - 1, 8
    bounds, ws = np.zeros(n + 1, np.int32), np.zeros(n, np.int64)
    pieces, xfers = (_lib.Piece * 64)(), (_lib.Xfer * 1024)()
    npc, nx = ctypes.c_int32(0), ctypes.c_int32(0)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)

    def med(flags):
        ts = []
        for _ in range(31):
            t0 = time.perf_counter()
            st = lib.tgms_multi_schedule(n, B, ptr(so), 0, flags, ptr(bounds), ptr(ws), pieces, 64,
                                         ctypes.byref(npc), xfers, 1024, ctypes.byref(nx))
            ts.append(time.perf_counter() - t0)
            assert st == 0
        return sorted(ts)[15]
    refine = med(REFINE | 4 | 8 | 16)
    solve = med(SOLVE | 4 | 8)

    def med_m(flags, so_, method):
        ts = []
        for _ in range(11):
            t0 = time.perf_counter()
            st = lib.tgms_multi_schedule(n, len(so_) - 1, ptr(so_), method, flags, ptr(bounds), ptr(ws), pieces, 64,
                                         ctypes.byref(npc), xfers, 1024, ctypes.byref(nx))
            ts.append(time.perf_counter() - t0)
            assert st == 0
        return sorted(ts)[5]
    band = med_m(SOLVE | 4 | 8, so, 2)
    uni = med_m(SOLVE | 4 | 8, SY.uniform_batch(1 << 20, 10)[0].astype(np.int32), 0)
    print(f"tgms_multi_schedule n=8 B=1,048,576 ragged: refinement loop {refine * 1e3:.4f} ms, reduced solve "
          f"{solve * 1e3:.4f} ms ({npc.value} pieces, {nx.value} transfers); band solve (validation pass) "
          f"{band * 1e3:.3f} ms; uniform M=10 reduced solve (uniform detection) {uni * 1e3:.3f} ms")
    assert refine <= 1e-4
    assert solve <= 1e-4
