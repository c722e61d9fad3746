"""Synthetic waypoint batches exactly as SURVEY.md §8(d) specifies them.

* seed 20251015, numpy PCG64 (``np.random.default_rng``);
* waypoints i.i.d. uniform in the reference room bounds: x, y in [-5, 5]
  (config/default.yaml:68-71), z in [0.5, 5.0] (kept above ground, within
  z_min/z_max :72-73);
* segment times T_i = clip(|w_{i+1} - w_i| / v, 0.5, 10) s with v = 1.0 m/s
  (v_line, config/default.yaml:51);
* rest-to-rest ends (every reference primitive starts and ends at rest).
"""
from __future__ import annotations

import numpy as np

SEED = 20251015
V_NOMINAL = 1.0
T_MIN, T_MAX = 0.5, 10.0


def _times(W: np.ndarray) -> np.ndarray:
    d = np.linalg.norm(np.diff(W, axis=-2), axis=-1)
    return np.clip(d / V_NOMINAL, T_MIN, T_MAX)


def uniform_batch(B: int, M: int, seed: int = SEED):
    """B trajectories of M segments: (seg_offsets [B+1], waypoints [B,M+1,3], times [B,M])."""
    rng = np.random.default_rng(seed)
    W = np.empty((B, M + 1, 3), dtype=np.float64)
    W[..., 0] = rng.uniform(-5.0, 5.0, size=(B, M + 1))
    W[..., 1] = rng.uniform(-5.0, 5.0, size=(B, M + 1))
    W[..., 2] = rng.uniform(0.5, 5.0, size=(B, M + 1))
    T = _times(W)
    so = (np.arange(B + 1, dtype=np.int64) * M).astype(np.int32)
    return so, W, T


def ragged_batch(B: int, m_lo: int = 2, m_hi: int = 16, seed: int = SEED):
    """Config 5: M_b ~ U{m_lo..m_hi}.  Returns CSR (seg_offsets, waypoints [S+B,3], times [S])."""
    rng = np.random.default_rng(seed)
    Ms = rng.integers(m_lo, m_hi + 1, size=B).astype(np.int32)
    so = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(Ms, out=so[1:])
    S = int(so[-1])
    n_w = S + B
    W = np.empty((n_w, 3), dtype=np.float64)
    W[:, 0] = rng.uniform(-5.0, 5.0, size=n_w)
    W[:, 1] = rng.uniform(-5.0, 5.0, size=n_w)
    W[:, 2] = rng.uniform(0.5, 5.0, size=n_w)
    # segment i of trajectory b joins waypoint rows so[b]+b+i and +1
    rows = np.arange(S) + np.repeat(np.arange(B), Ms)
    T = np.clip(np.linalg.norm(W[rows + 1] - W[rows], axis=1) / V_NOMINAL, T_MIN, T_MAX)
    return so.astype(np.int32), W, T
