"""Device entry points inside a caller's HIP-graph capture.

bench.py captures the uniform reduced solve into one graph of K steps.  The handle's
scratch handshake (an event recorded on the caller's stream) cannot order the replays
of a captured graph, so inside a capture the library skips it, and every call that
would upload a host-side launch plan or grow device scratch at call time (ragged
batches, the refinement loop, multi-GPU calls, a band slab that must grow) refuses
with TGMS_ERR_UNSUPPORTED instead of capturing a plan the handle later overwrites.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _capture(fn):
    """Run fn(stream) under torch.cuda.graph capture on a side stream; return the graph
    (or None) and the exception fn raised, if any (caught inside the capture so the
    capture itself ends normally)."""
    import torch
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    err = None
    with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
        try:
            fn(side.cuda_stream)
        except Exception as e:  # noqa: BLE001 -- reported to the caller
            err = e
    torch.cuda.current_stream().wait_stream(side)
    return g, err


@pytest.mark.parametrize("meth", ["reduced", "band", "dense"])
def test_uniform_solve_captured_and_replayed(solver, meth):
    import torch
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_DENSE_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    m = {"reduced": METHOD_REDUCED, "band": METHOD_BAND_KKT, "dense": METHOD_DENSE_KKT}[meth]
    B, M = 4096, 7
    _, W, T = S.uniform_batch(B, M, seed=90)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    solver.set_method(m)
    try:
        ref = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
        solver.solve_uniform_device(B, M, dW, dT, ref)  # (grows the band slab outside the capture)
        torch.cuda.synchronize()
        out = torch.full_like(ref, float("nan"))
        st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        g, err = _capture(lambda s: solver.solve_uniform_device(B, M, dW, dT, out, st, stream=s))
        assert err is None, err
        torch.cuda.synchronize()
        for _ in range(3):
            out.fill_(float("nan"))
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out, ref)
            assert int(st.abs().sum()) == 0
        del g
    finally:
        solver.set_method(METHOD_REDUCED)


def test_ragged_and_loop_calls_refuse_capture(solver):
    import torch
    from trajectory_generator_ros2_amd import ERR_UNSUPPORTED, TgmsError
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(500, 2, 9, seed=91)
    d = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    dso, dW, dT = d(so), d(W), d(T.copy())
    S_ = int(so[-1])
    C = torch.empty((S_, 3, 8), dtype=torch.float64, device="cuda")
    calls = [lambda s: solver.solve_batch_device(so, dso, dW, dT, C, stream=s),
             lambda s: solver.refine_loop_device(so, dso, dW, dT, 1.0, 0.1, 3, C, stream=s)]
    for fn in calls:
        _, err = _capture(fn)
        assert isinstance(err, TgmsError) and err.status == ERR_UNSUPPORTED, err
        assert "capture" in solver.last_error()
    # the handle works normally afterwards, and matches the host API
    solver.solve_batch_device(so, dso, dW, dT, C)
    torch.cuda.synchronize()
    Ch, _, worst = solver.solve(so, W, T)
    assert worst == 0 and np.array_equal(C.cpu().numpy(), Ch)


def test_band_graph_keeps_its_slab_when_the_handle_grows():
    """a captured band-KKT launch bakes in the slab pointer.  Once a capture
    has used a slab it belongs to graphs: an uncaptured call that needs a bigger slab
    allocates its own (the graph's is never freed under it), and an uncaptured call
    running beside a replay uses a different slab.  Capture, grow, replay (also
    concurrently with uncaptured calls on another stream): every result exact."""
    import torch
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import Solver
    B = 4096
    data = {}
    for M in (3, 16):
        _, W, T = S.uniform_batch(B, M, seed=92 + M)
        data[M] = (torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda())
    with Solver(0) as s:
        ref = {}
        for M in (3, 16):  # the reduced solve as the reference
            ref[M] = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
            s.solve_uniform_device(B, M, *data[M], ref[M])
        s.set_method(METHOD_BAND_KKT)
        out3 = torch.empty_like(ref[3])
        s.solve_uniform_device(B, 3, *data[3], out3)  # slab for M = 3
        torch.cuda.synchronize()
        g, err = _capture(lambda st: s.solve_uniform_device(B, 3, *data[3], out3, stream=st))
        assert err is None, err
        out16 = torch.empty_like(ref[16])
        s.solve_uniform_device(B, 16, *data[16], out16)  # grows: a new slab, the graph's stays
        torch.cuda.synchronize()
        tol = lambda a, b: float(((a - b).abs().amax(dim=(1, 3)) / b.abs().amax(dim=(1, 3))).max())
        assert tol(out16, ref[16]) <= 1e-9
        other = torch.cuda.Stream()
        for _ in range(3):
            out3.fill_(float("nan"))
            out16.fill_(float("nan"))
            g.replay()  # on the current stream
            with torch.cuda.stream(other):  # beside it, uncaptured, on the handle's own slab
                s.solve_uniform_device(B, 16, *data[16], out16, stream=other.cuda_stream)
            torch.cuda.synchronize()
            assert tol(out3, ref[3]) <= 1e-9
            assert tol(out16, ref[16]) <= 1e-9
        del g
        s.set_method(METHOD_REDUCED)


def test_band_capture_waits_for_an_uncaptured_call_in_flight():
    """the first capture of a band-KKT call takes over the handle's slab.  An
    uncaptured call still running on that slab (another stream, not synchronised) must be
    finished before any replay can use it: the hand-off waits for the handle's last
    uncaptured user.  Uncaptured call in flight -> capture -> immediate replay: both exact."""
    import torch
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import Solver
    M, Bbig, B = 16, 65536, 4096
    _, Wb, Tb = S.uniform_batch(Bbig, M, seed=301)
    _, W, T = S.uniform_batch(B, M, seed=302)
    dWb, dTb = torch.from_numpy(Wb).cuda(), torch.from_numpy(Tb).cuda()
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    with Solver(0) as s:
        refb = torch.empty((Bbig, M, 3, 8), dtype=torch.float64, device="cuda")
        ref = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
        s.solve_uniform_device(Bbig, M, dWb, dTb, refb)  # reduced solve: the reference
        s.solve_uniform_device(B, M, dW, dT, ref)
        torch.cuda.synchronize()
        s.set_method(METHOD_BAND_KKT)
        outb = torch.full_like(refb, float("nan"))
        out = torch.full_like(ref, float("nan"))
        other = torch.cuda.Stream()
        with torch.cuda.stream(other):  # ~2.5 ms of band work on the handle's slab, not waited for
            s.solve_uniform_device(Bbig, M, dWb, dTb, outb, stream=other.cuda_stream)
        g, err = _capture(lambda st: s.solve_uniform_device(B, M, dW, dT, out, stream=st))
        assert err is None, err
        g.replay()
        torch.cuda.synchronize()
        tol = lambda a, b: float(((a - b).abs().amax(dim=(1, 3)) / b.abs().amax(dim=(1, 3))).max())
        assert tol(outb, refb) <= 1e-9
        assert tol(out, ref) <= 1e-9
        del g
