"""Shared fixtures.  `-m gpu` tests need a HIP device and go through libtgms's C ABI;
everything else runs on CPU (oracle vs goldens, host logic, ABI exports, gloo)."""
import os

os.environ.setdefault("TGMS_NODE_QUIET", "1")  # the node adapter logs every generation (as the reference does)
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


def _deriv(c, t, k):
    """k-th derivative of sum_j c_j t^j (c [..., 8], t broadcastable to c[..., 0])."""
    j = np.arange(8)
    f = np.array([np.prod(np.arange(jj - k + 1, jj + 1)) if jj >= k else 0.0 for jj in j])
    p = np.where(j >= k, j - k, 0)
    return (c * f * np.power(np.asarray(t)[..., None], p)).sum(-1)


def check_spline_properties(so, W, T, C, atol_pos=1e-8, rtol_cont=1e-7):
    """Size-independent properties of a rest-to-rest min-snap solution of a CSR batch
    (every trajectory, any size): c0 = start waypoint and p(T) = end waypoint of every
    segment, derivatives 1..6 continuous at every interior knot, v = a = j = 0 at both
    ends.  so [B+1], W [S+B,3], T [S], C [S,3,8]."""
    so = np.asarray(so, dtype=np.int64)
    B = so.shape[0] - 1
    S = int(so[-1])
    W = np.asarray(W).reshape(-1, 3)
    T = np.asarray(T).reshape(-1)
    C = np.asarray(C).reshape(S, 3, 8)
    Ms = np.diff(so)
    traj = np.repeat(np.arange(B), Ms)
    rows = np.arange(S) + traj                     # start waypoint row of every segment
    np.testing.assert_allclose(C[..., 0], W[rows], rtol=0, atol=1e-12)
    Tt = np.repeat(T[:, None], 3, axis=1)          # [S,3]
    np.testing.assert_allclose(_deriv(C, Tt, 0), W[rows + 1], rtol=0, atol=atol_pos)
    first = so[:-1]
    last = so[1:] - 1
    inner = np.setdiff1d(np.arange(S - 1), last)  # segment s and s+1 in one trajectory
    for k in range(1, 7):
        left = _deriv(C[inner], Tt[inner], k)
        right = _deriv(C[inner + 1], 0.0 * Tt[inner + 1], k)
        scale = np.abs(right).max() + 1.0 if right.size else 1.0
        assert np.abs(left - right).max(initial=0.0) <= rtol_cont * scale, k
    for k in range(1, 4):
        assert np.abs(C[first, :, k]).max() == 0.0
        assert np.abs(_deriv(C[last], Tt[last], k)).max() <= atol_pos



def check_spline_properties_torch(so, W, T, C, atol_pos=1e-8, rtol_cont=1e-7, chunk=1 << 20):
    """check_spline_properties for a batch held in torch tensors (fp64, any device:
    the 1,048,576-trajectory configs are checked where they live).  Same properties
    and tolerances: c0 = start waypoint (1e-12), p(T) = end waypoint (atol_pos),
    derivatives 1..6 continuous at every interior knot (rtol_cont x (max|right| + 1)
    over a chunk of `chunk` segments), v = a = j = 0 at both ends.  Plain torch
    elementwise arithmetic, independent of the kernels under test."""
    import torch
    dev = C.device
    so = torch.as_tensor(np.asarray(so, dtype=np.int64), device=dev)
    W = W.reshape(-1, 3)
    T = T.reshape(-1)
    C = C.reshape(-1, 3, 8)
    B = so.numel() - 1
    S = C.shape[0]
    Ms = so[1:] - so[:-1]
    rows = torch.arange(S, device=dev) + torch.repeat_interleave(torch.arange(B, device=dev), Ms)
    last = torch.zeros(S, dtype=torch.bool, device=dev)
    last[so[1:] - 1] = True
    first = so[:-1]
    assert float((C[..., 0] - W[rows]).abs().max()) <= 1e-12
    assert float(C[first][:, :, 1:4].abs().max()) == 0.0
    j = torch.arange(8, device=dev, dtype=torch.float64)
    fact = [1.0, 1.0, 2.0, 6.0, 24.0, 120.0, 720.0]
    for s0 in range(0, S, chunk):
        s1 = min(S, s0 + chunk)
        t = T[s0:s1, None]
        cs = C[s0:s1]
        inner = ~last[s0:s1]
        if s1 == S:
            inner[-1] = False
        nxt = C[s0 + 1:min(S, s1 + 1)]
        for k in range(0, 7):
            f = torch.ones(8, device=dev, dtype=torch.float64)
            for q in range(k):
                f = f * (j - q)
            f = torch.where(j >= k, f, torch.zeros_like(f))
            G = f * torch.pow(t, torch.clamp(j - k, min=0))  # [n, 8]
            val = (cs * G[:, None, :]).sum(-1)               # [n, 3]: k-th derivative at T
            if k == 0:
                assert float((val - W[rows[s0:s1] + 1]).abs().max()) <= atol_pos
                continue
            if 1 <= k <= 3:
                lv = val[last[s0:s1]]
                assert lv.numel() == 0 or float(lv.abs().max()) <= atol_pos, k
            n_in = int(inner.sum())
            if n_in:
                idx = torch.nonzero(inner).reshape(-1)
                right = fact[k] * nxt[idx][:, :, k]
                left = val[idx]
                scale = float(right.abs().max()) + 1.0
                assert float((left - right).abs().max()) <= rtol_cont * scale, k


def check_spline_properties_chunked(so, W, T, C, chunk=65536, **kw):
    """check_spline_properties over a large CSR batch in host chunks of `chunk`
    trajectories (every trajectory is checked; the temporaries stay ~chunk-sized)."""
    so = np.asarray(so, dtype=np.int64)
    W = np.asarray(W).reshape(-1, 3)
    T = np.asarray(T).reshape(-1)
    C = np.asarray(C).reshape(-1, 3, 8)
    B = so.shape[0] - 1
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        s0, s1 = int(so[lo]), int(so[hi])
        check_spline_properties(so[lo:hi + 1] - s0, W[s0 + lo:s1 + hi + 1], T[s0:s1], C[s0:s1], **kw)


REFINE_GROUPS = ("u10", "u10e", "u7e", "u16", "r", "re", "u257", "u257e", "r257", "r257e")


def load_refine_golden():
    """tests/golden/refine_grad.npz (exact config-5 step, make_golden.py): returns
    (k_T, eta, {group: dict(seg_offsets, waypoints, seg_times, end_derivs|None, J, dJ, F, T1)})."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "refine_grad.npz"))
    groups = {}
    for g in REFINE_GROUPS:
        d = {k: z[g + "_" + k] for k in ("seg_offsets", "waypoints", "seg_times", "J", "dJ", "F", "T1")}
        d["end_derivs"] = z[g + "_end_derivs"] if (g + "_end_derivs") in z.files else None
        groups[g] = d
    return float(z["k_T"]), float(z["eta"]), groups


def recovered_gradient(T0, T1, F0, k_T, eta):
    """The per-segment dJ_i/dT_i a refinement step applied, recovered from its output:
    T1 = T0 exp(-eta T0 (dJ + k_T) / F0)  =>  dJ = -log(T1/T0) F0 / (eta T0) - k_T.
    Also returns the mask of unclamped segments (|dtau| < 1/2)."""
    dtau = np.log(np.asarray(T1) / np.asarray(T0))
    return -dtau * F0 / (eta * T0) - k_T, np.abs(dtau) < 0.499


def gradient_rel_err(so, g, ref, mask=None):
    """Worst per-trajectory norm-wise error max_i |g_i - ref_i| / max_i |ref_i| over a CSR
    batch (segments outside `mask` are skipped in the numerator)."""
    so = np.asarray(so, dtype=np.int64)
    d = np.abs(np.asarray(g) - np.asarray(ref))
    if mask is not None:
        d = np.where(mask, d, 0.0)
    num = np.maximum.reduceat(d, so[:-1])
    den = np.maximum.reduceat(np.abs(ref), so[:-1])
    return float((num / np.where(den == 0.0, 1.0, den)).max())


def solve_goldens():
    """The solve fixtures of tests/golden (every *.npz except the refinement step's)."""
    import glob
    return sorted(p for p in glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz"))
                  if os.path.basename(p) != "refine_grad.npz")
