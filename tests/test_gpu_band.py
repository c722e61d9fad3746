"""GPU parity of TGMS_METHOD_BAND_KKT (tgms_band.hip): the survey's literal KKT, LU with
partial pivoting in the segment-interleaved order, against the oracle's dense GEPP of
the same permuted matrix (oracle KKT_BAND), the other formulations and the exact
goldens.  Tolerance as everywhere: norm-wise per (trajectory, axis) <= 1e-9."""
import os

import numpy as np
import pytest

from conftest import batch_rel_err, solve_goldens

pytestmark = pytest.mark.gpu

TOL = 1e-9
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture
def band(solver):
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_REDUCED
    solver.set_method(METHOD_BAND_KKT)
    yield solver
    solver.set_method(METHOD_REDUCED)


def _uniform(B, M, seed):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(B, M, seed=seed)
    return so, W.reshape(-1, 3), T.reshape(-1)


@pytest.mark.parametrize("M", list(range(1, 17)))
def test_band_uniform_vs_oracle(band, oracle, M):
    so, W, T = _uniform(129, M, seed=900 + M)  # odd: the last wavefront has one dead half
    C, st, worst = band.solve(so, W, T)
    assert worst == 0 and (st == 0).all()
    R, rst = oracle.solve_batch(so, W, T, None, oracle.KKT_BAND)
    assert (rst == 0).all()
    assert batch_rel_err(so, C, R) <= TOL
    R2, _ = oracle.solve_batch(so, W, T, None, oracle.REDUCED)
    assert batch_rel_err(so, C, R2) <= TOL


def test_band_persistent_grid_reuses_slabs(band, oracle):
    """More trajectory pairs than wavefronts in the persistent grid (16 per CU): every
    wavefront solves several pairs through the same U slab."""
    so, W, T = _uniform(20001, 3, seed=910)
    C, st, worst = band.solve(so, W, T)
    assert worst == 0 and (st == 0).all()
    R, _ = oracle.solve_batch(so, W, T, None, oracle.KKT_BAND)
    assert batch_rel_err(so, C, R) <= TOL


def test_band_end_derivs(band, oracle):
    rng = np.random.default_rng(911)
    so, W, T = _uniform(101, 7, seed=911)
    ED = rng.normal(size=(101, 18))
    C, st, worst = band.solve(so, W, T, ED)
    assert worst == 0
    R, _ = oracle.solve_batch(so, W, T, ED, oracle.KKT_BAND)
    assert batch_rel_err(so, C, R) <= TOL


def test_band_ragged(band, oracle):
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(777, 1, 16, seed=912)
    C, st, worst = band.solve(so, W, T)
    assert worst == 0 and (st == 0).all()
    R, _ = oracle.solve_batch(so, W, T, None, oracle.REDUCED)
    assert batch_rel_err(so, C, R) <= TOL


@pytest.mark.parametrize("path", solve_goldens())
def test_band_goldens_exact(band, path):
    g = np.load(path)
    so = g["seg_offsets"]
    ED = g["end_derivs"] if "end_derivs" in g.files else None
    C, st, worst = band.solve(so, g["waypoints"], g["seg_times"], ED)
    assert worst == 0
    assert batch_rel_err(so, C, g["coeffs"]) <= TOL


def test_band_invalid_inputs(band):
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG
    so, W, T = _uniform(70, 4, seed=7)
    T = T.copy(); W = W.copy()
    T[4 * 3 + 1] = 0.0
    T[4 * 5] = -1.0
    W[(4 + 1) * 9 + 2, 1] = np.nan
    T[4 * 66 + 3] = np.inf
    C, st, worst = band.solve(so, W, T)
    bad = {3, 5, 9, 66}
    assert worst == ERR_INVALID_ARG
    assert all(st[b] == ERR_INVALID_ARG for b in bad)
    assert all(st[b] == 0 for b in range(70) if b not in bad)
    assert np.isfinite(C).all()
    assert all(not C[4 * b:4 * b + 4].any() for b in bad)


def test_band_config3_device_matches_reduced(band):
    """Config 3 at full size (65,536 x M = 10) through the device API: the band KKT and
    the reduced solve agree to the tolerance on every trajectory."""
    import torch
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    B, M = 65536, 10
    _, W, T = S.uniform_batch(B, M)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    dC = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
    dR = torch.empty_like(dC)
    dS = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    band.solve_uniform_device(B, M, dW, dT, dC, dS)
    band.set_method(METHOD_REDUCED)
    band.solve_uniform_device(B, M, dW, dT, dR, None)
    band.set_method(METHOD_BAND_KKT)
    torch.cuda.synchronize()
    assert int((dS != 0).sum()) == 0
    err = (dC - dR).abs().amax(dim=(1, 3)) / dR.abs().amax(dim=(1, 3))
    assert float(err.max()) <= TOL


@pytest.mark.parametrize("B,M,seed", [(131072, 16, 7000), (131072, 16, 1), (40000, 16, 7000),
                                      (131072, 10, 7000), (40000, 10, 7000), (40000, 3, 910)])
def test_band_slab_reuse_at_round3_failing_shapes(band, oracle, B, M, seed):
    """The shapes at which round 3's two-wave build returned wrong coefficients with status
    OK (scripts/band_diag.py): every wavefront of the persistent grid solves
    several 16-trajectory groups through its one U slab.  The shipped build, twice (the
    failures varied run to run): every trajectory against the reduced solve, slices at the
    start, the middle and the end against the oracle's dense GEPP (KKT_BAND)."""
    import torch
    from trajectory_generator_ros2_amd import METHOD_BAND_KKT, METHOD_REDUCED
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.uniform_batch(B, M, seed=seed)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    dR = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
    band.set_method(METHOD_REDUCED)
    band.solve_uniform_device(B, M, dW, dT, dR, None)
    band.set_method(METHOD_BAND_KKT)
    dC = torch.empty_like(dR)
    dS = torch.empty((B,), dtype=torch.int32, device="cuda")
    for rep in range(2):
        dC.fill_(np.nan)
        dS.fill_(-1)
        band.solve_uniform_device(B, M, dW, dT, dC, dS)
        torch.cuda.synchronize()
        assert int((dS != 0).sum()) == 0, rep
        err = (dC - dR).abs().amax(dim=(1, 3)) / dR.abs().amax(dim=(1, 3))
        nbad = int((~(err <= TOL)).sum())
        assert nbad == 0, (rep, nbad, float(err.max()))
    Wf, Tf = W.reshape(B, M + 1, 3), T.reshape(B, M)
    C = dC.cpu().numpy()
    for lo in (0, B // 2 - 128, B - 256):
        sl = slice(lo, lo + 256)
        so_s = np.arange(257, dtype=np.int32) * M
        R, rst = oracle.solve_batch(so_s, Wf[sl].reshape(-1, 3), Tf[sl].reshape(-1), None, oracle.KKT_BAND)
        assert (rst == 0).all()
        assert batch_rel_err(so_s, C[sl].reshape(-1, 3, 8), R) <= TOL


def test_band_ragged_end_derivs_and_invalid(band, oracle):
    """A ragged batch (every M in 1..16, groups solved one after another through the
    shared U slabs) with end derivatives and invalid trajectories in several groups:
    valid ones match the oracle, invalid ones are flagged and zeroed."""
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG
    from trajectory_generator_ros2_amd import synthetic as S
    rng = np.random.default_rng(913)
    so, W, T = S.ragged_batch(600, 1, 16, seed=913)
    B = len(so) - 1
    ED = rng.normal(size=(B, 18))
    T = T.copy()
    M = np.diff(so)
    bad = [int(np.flatnonzero(M == m)[0]) for m in (1, 6, 11, 16)]
    for b in bad:
        T[so[b]] = 0.0
    C, st, worst = band.solve(so, W, T, ED)
    assert worst == ERR_INVALID_ARG
    assert all(st[b] == ERR_INVALID_ARG for b in bad)
    good = np.setdiff1d(np.arange(B), bad)
    assert (st[good] == 0).all()
    for b in bad:
        assert not C[so[b]:so[b + 1]].any()
    T2 = T.copy()
    for b in bad:
        T2[so[b]] = 1.0
    R, _ = oracle.solve_batch(so, W, T2, ED, oracle.KKT_BAND)
    for b in good:
        c, r = C[so[b]:so[b + 1]], R[so[b]:so[b + 1]]
        for a in range(3):
            assert np.abs(c[:, a] - r[:, a]).max() <= TOL * max(np.abs(r[:, a]).max(), 1e-300)
