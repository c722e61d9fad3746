"""The property checker the full-size GPU tests use (conftest.check_spline_properties_torch)
agrees with the numpy one on an oracle solution and catches single perturbations of
every property it claims (CPU torch)."""
import numpy as np
import pytest

from conftest import check_spline_properties, check_spline_properties_torch


def test_torch_checker_accepts_and_rejects(oracle):
    import torch
    from trajectory_generator_ros2_amd import synthetic as S
    so, W, T = S.ragged_batch(3000, 1, 16, seed=12)
    C, st = oracle.solve_batch(so, W, T, None, oracle.REDUCED, 4)
    assert (st == 0).all()
    check_spline_properties(so, W, T, C)
    t = torch.from_numpy
    check_spline_properties_torch(so, t(W), t(T), t(C), chunk=4096)
    # interior knot (continuity k = 3), last segment (end rest / interpolation),
    # first segment (rest start: exact zero), start waypoint (c0)
    for seg, ax, k, d in [(100, 0, 3, 1e-6), (int(so[7]) - 1, 1, 5, 1e-3), (int(so[9]), 2, 1, 1e-12),
                          (int(so[11]) - 1, 0, 7, 1e-6), (int(so[20]) + 1, 1, 0, 1e-9)]:
        C2 = C.copy()
        C2[seg, ax, k] += d
        with pytest.raises(AssertionError):
            check_spline_properties_torch(so, t(W), t(T), t(C2), chunk=4096)
