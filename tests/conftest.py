"""Shared fixtures.  `-m gpu` tests need a HIP device and go through libtgms's C ABI;
everything else runs on CPU (oracle vs goldens, host logic, ABI exports, gloo)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs through libtgms")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    if not os.path.exists(O.LIB_PATH):
        O.build()
    return O


@pytest.fixture(scope="session")
def solver():
    from trajectory_generator_ros2_amd.build import LIB_TGMS, build_tgms
    from trajectory_generator_ros2_amd.solver import Solver
    if not os.path.exists(LIB_TGMS):
        build_tgms()
    s = Solver(0)
    yield s
    s.close()


def normwise_rel_err(C, R):
    """max over (trajectory-segment-block, axis) of ||dC||_inf / ||R||_inf, per SURVEY.md §8(c).
    C, R: [S,3,8] for one trajectory (or a list of per-trajectory arrays)."""
    C = np.asarray(C, dtype=np.float64)
    R = np.asarray(R, dtype=np.float64)
    num = np.abs(C - R).max(axis=(0, 2))
    den = np.abs(R).max(axis=(0, 2))
    den = np.where(den == 0.0, 1.0, den)
    return float((num / den).max())


def batch_rel_err(so, C, R):
    """Worst per-(trajectory, axis) norm-wise relative error over a CSR batch."""
    so = np.asarray(so, dtype=np.int64)
    C = np.asarray(C, dtype=np.float64).reshape(-1, 3, 8)
    R = np.asarray(R, dtype=np.float64).reshape(-1, 3, 8)
    d = np.abs(C - R).max(axis=2)
    r = np.abs(R).max(axis=2)
    dm = np.maximum.reduceat(d, so[:-1], axis=0)
    rm = np.maximum.reduceat(r, so[:-1], axis=0)
    rm = np.where(rm == 0.0, 1.0, rm)
    return float((dm / rm).max())
