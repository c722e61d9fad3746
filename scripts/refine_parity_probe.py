"""Measure the config-5 refinement parity figures on the GPU (one JSON line per check).

- exact fixture (tests/golden/refine_grad.npz): GPU F(T_0), T_1 and the applied gradient
  vs exact arithmetic, and the fp64 oracle's the same way;
- 257-trajectory one-step cases (test_gpu_parity.py): GPU gradient vs the oracle's;
- 10 steps (k_T 1, eta 0.1): GPU vs oracle times / costs, 257 uniform + ragged, and three
  1,024-trajectory slices of config 5's per-GPU share.
    python scripts/refine_parity_probe.py > gpurun_out/refine_probe.jsonl
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import gradient_rel_err, load_refine_golden, recovered_gradient  # noqa: E402
from oracle import oracle as O  # noqa: E402
from trajectory_generator_ros2_amd import shard as SH  # noqa: E402
from trajectory_generator_ros2_amd import synthetic as S  # noqa: E402
from trajectory_generator_ros2_amd.solver import Solver  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    s = Solver(0)
    k_T, eta, groups = load_refine_golden()
    for g, d in groups.items():
        so, W, T, ED = d["seg_offsets"], d["waypoints"], d["seg_times"], d["end_derivs"]
        _, _, F0, _, w0 = s.refine(so, W, T, ED, k_T, eta, 0, coeffs=False)
        T1, _, _, _, w1 = s.refine(so, W, T, ED, k_T, eta, 1, coeffs=False)
        gg, free = recovered_gradient(T, T1, np.repeat(F0, np.diff(so)), k_T, eta)
        To, Fo, _, _ = O.refine_batch(so, W, T, ED, k_T, eta, 1, O.REDUCED)
        _, Fo0, _, _ = O.refine_batch(so, W, T, ED, k_T, eta, 0, O.REDUCED)
        go, fo = recovered_gradient(T, To, np.repeat(Fo0, np.diff(so)), k_T, eta)
        emit(check="exact_fixture", group=g, worst=int(max(w0, w1)),
             gpu_F0=float(np.abs(F0 / d["F"] - 1).max()), gpu_T1=float(np.abs(T1 / d["T1"] - 1).max()),
             gpu_grad=gradient_rel_err(so, gg, d["dJ"], free),
             oracle_T1=float(np.abs(To / d["T1"] - 1).max()), oracle_grad=gradient_rel_err(so, go, d["dJ"], fo))
    for ragged in (False, True):
        for with_ed in (False, True):
            if ragged:
                so, W, T = S.ragged_batch(257, 1, 16, seed=61)
            else:
                so, W, T = S.uniform_batch(257, 10, seed=62)
            W, T = W.reshape(-1, 3), T.reshape(-1)
            B = len(so) - 1
            ED = np.random.default_rng(63).normal(scale=0.3, size=(B, 18)) if with_ed else None
            _, _, F0, _, _ = s.refine(so, W, T, ED, 1.0, 0.02, 0, coeffs=False)
            T1, _, _, _, _ = s.refine(so, W, T, ED, 1.0, 0.02, 1, coeffs=False)
            dJ = np.zeros_like(T)
            for b in range(B):
                s0, s1 = int(so[b]), int(so[b + 1])
                dJ[s0:s1] = O.refine_grad(W[s0 + b:s1 + b + 1], T[s0:s1], None if ED is None else ED[b], 1.0,
                                          O.REDUCED)[0]
            g, free = recovered_gradient(T, T1, np.repeat(F0, np.diff(so)), 1.0, 0.02)
            emit(check="one_step_vs_oracle", ragged=ragged, with_ed=with_ed,
                 grad=gradient_rel_err(so, g, dJ, free))
            Tg, _, cg, _, _ = s.refine(so, W, T, ED, 1.0, 0.1, 10, coeffs=False)
            To, co, _, _ = O.refine_batch(so, W, T, ED, 1.0, 0.1, 10, O.REDUCED)
            emit(check="ten_steps_vs_oracle", ragged=ragged, with_ed=with_ed,
                 T=float(np.abs(Tg / To - 1).max()), cost=float(np.abs(cg / co - 1).max()))
    so_all, W_all, T_all = S.ragged_batch(1048576, 2, 16)
    bounds = SH.ragged_bounds(so_all, 8)
    so, W, T, _ = SH.shard_csr(so_all, W_all, T_all, None, int(bounds[0]), int(bounds[1]))
    B = len(so) - 1
    Tg, _, cg, _, _ = s.refine(so, W, T, None, 1.0, 0.1, 10, coeffs=False)
    dT, dc = [], []
    for lo, hi in [(0, 1024), (B // 2 - 512, B // 2 + 512), (B - 1024, B)]:
        so_l, W_l, T_l, _ = SH.shard_csr(so, W, T, None, lo, hi)
        To, co, _, _ = O.refine_batch(so_l, W_l, T_l, None, 1.0, 0.1, 10, O.REDUCED)
        s0, s1 = int(so[lo]), int(so[hi])
        dT.append(np.abs(Tg[s0:s1] / To - 1))
        dc.append(np.abs(cg[lo:hi] / co - 1))
    dT, dc = np.concatenate(dT), np.concatenate(dc)
    emit(check="config5_share_slices", T_max=float(dT.max()), T_p99=float(np.quantile(dT, 0.99)),
         cost_max=float(dc.max()), cost_p99=float(np.quantile(dc, 0.99)))
    s.close()


if __name__ == "__main__":
    main()
