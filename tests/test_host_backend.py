"""CPU: the explicit host backend of the C ABI (tgms_create_host; csrc/tgms_host.cpp).

BASELINE config 1 is "single goal, 3-segment order-7 min-snap, 3 axes via CPU
TrajectoryGenerator (ROS2 node up, no GPU)": the reference generates on the executor
thread's CPU (src/TrajectoryGenerator.cpp:54-57, :71).  A GPU-less node asks for this
backend explicitly (`minsnap_backend: host`); tgms_create never falls back to it
(tests/test_node_host.py::test_no_cpu_fallback).  Its solve is the product's own reduced
formulation, held here to the oracle and the exact goldens at north_star's
1e-9 (norm-wise per trajectory and axis), its sampler to the oracle's."""
import os

import numpy as np
import pytest

from conftest import batch_rel_err, solve_goldens

TOL = 1e-9
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def host():
    from trajectory_generator_ros2_amd.build import LIB_TGMS, build_tgms
    from trajectory_generator_ros2_amd.solver import Solver
    if not os.path.exists(LIB_TGMS):
        build_tgms()
    s = Solver(host=True)
    yield s
    s.close()


@pytest.mark.parametrize("M", list(range(1, 17)))
@pytest.mark.parametrize("with_ed", [False, True])
def test_host_solve_vs_oracle(host, oracle, M, with_ed):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(64, M, seed=500 + M)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    ED = np.random.default_rng(M).normal(size=(64, 18)) if with_ed else None
    C, st, worst = host.solve(so, W, T, ED)
    assert worst == 0 and (st == 0).all()
    R, rst = oracle.solve_batch(so, W, T, ED, oracle.KKT_C4 if M <= 10 else oracle.REDUCED)
    assert (rst == 0).all()
    assert batch_rel_err(so, C, R) <= TOL


def test_host_ragged_vs_oracle(host, oracle):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(500, 1, 16, seed=77)
    C, st, worst = host.solve(so, W, T)
    assert worst == 0
    R, _ = oracle.solve_batch(so, W, T, None, oracle.REDUCED)
    assert batch_rel_err(so, C, R) <= TOL


@pytest.mark.parametrize("path", solve_goldens())
def test_host_goldens_exact(host, path):
    g = np.load(path)
    so = g["seg_offsets"]
    ED = g["end_derivs"] if "end_derivs" in g.files else None
    C, st, worst = host.solve(so, g["waypoints"], g["seg_times"], ED)
    assert worst == 0
    assert batch_rel_err(so, C, g["coeffs"]) <= TOL


def test_host_config1_sampled_vs_golden(host):
    """Config 1 end to end (4 waypoints, 3 segments, sampled at the reference's pub_freq)."""
    for name in ("c1", "c3_sampled"):
        g = np.load(os.path.join(GOLDEN, name + ".npz"))
        if "samples" not in g.files:
            continue
        so = g["seg_offsets"]
        ED = g["end_derivs"] if "end_derivs" in g.files else None
        C, _, worst = host.solve(so, g["waypoints"], g["seg_times"], ED)
        assert worst == 0
        offs, out = host.sample(so, g["waypoints"], g["seg_times"], ED, C, float(g["dt"]))
        assert np.array_equal(offs, g["sample_offsets"])
        ref = g["samples"]
        for f0, f1 in ((0, 3), (3, 6), (6, 9), (9, 12)):
            assert np.abs(out[:, f0:f1] - ref[:, f0:f1]).max() <= TOL * np.abs(ref[:, f0:f1]).max()


@pytest.mark.parametrize("yaw_mode", [0, 1])
def test_host_sample_vs_oracle(host, oracle, yaw_mode):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(6, 2, 9, seed=3)
    W, T = W.reshape(-1, 3), T.reshape(-1)
    ED = np.random.default_rng(4).normal(size=(6, 18))
    C, _, worst = host.solve(so, W, T, ED)
    assert worst == 0
    offs, out = host.sample(so, W, T, ED, C, 0.01, yaw_mode=yaw_mode, yaw_const=0.3)
    for b in range(6):
        s0, s1 = int(so[b]), int(so[b + 1])
        ref = oracle.sample(C[s0:s1], T[s0:s1], W[s0 + b:s1 + b + 1], ED[b], 0.01, yaw_mode, 0.3)
        got = out[offs[b]:offs[b + 1]]
        assert got.shape == ref.shape
        assert np.abs(got[:, :12] - ref[:, :12]).max() <= TOL * max(1.0, np.abs(ref[:, :12]).max())
        assert np.abs(np.angle(np.exp(1j * (got[:, 12] - ref[:, 12])))).max() <= 1e-9
        assert np.abs(got[:, 13] - ref[:, 13]).max() <= 1e-7 * max(1.0, np.abs(ref[:, 13]).max())


def test_host_invalid_inputs_are_zero(host):
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(4, 3, seed=1)
    W, T = W.reshape(-1, 3).copy(), T.reshape(-1).copy()
    T[4] = -1.0           # trajectory 1
    W[2 * 4 + 1, 0] = np.nan  # trajectory 2
    C, st, worst = host.solve(so, W, T, check=False)
    assert worst == ERR_INVALID_ARG
    assert list(st) == [0, ERR_INVALID_ARG, ERR_INVALID_ARG, 0]
    assert not C[3:9].any()


def test_host_handle_refuses_device_entry_points(host):
    import torch
    from trajectory_generator_ros2_amd import ERR_UNSUPPORTED, METHOD_BAND_KKT, TgmsError
    assert host.device_count == 0
    with pytest.raises(TgmsError) as e:
        host.set_method(METHOD_BAND_KKT)
    assert e.value.status == ERR_UNSUPPORTED
    dW = torch.zeros((4, 3), dtype=torch.float64)
    dT = torch.ones(3, dtype=torch.float64)
    dC = torch.zeros((3, 3, 8), dtype=torch.float64)
    with pytest.raises(TgmsError) as e:
        host.solve_uniform_device(1, 3, dW, dT, dC)
    assert e.value.status == ERR_UNSUPPORTED
    assert host.refine(np.array([0, 3], np.int32), dW.numpy(), dT.numpy(), None, 1.0, 0.1, 2)[-1] == ERR_UNSUPPORTED
