"""CPU: the C ABI's multi-GPU shard planner (tgms_plan_shards, include/tgms.h) gives the
same contiguous cost-balanced bounds as shard.ragged_bounds, the Python planner of the
torch.distributed path; argument checks; tgms_create_multi fails loudly with no GPU;
RCCL is not a link-time dependency (it is loaded by tgms_create_multi)."""
import subprocess

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    import os
    from trajectory_generator_ros2_amd import _lib
    from trajectory_generator_ros2_amd.build import LIB_TGMS, build_tgms
    if not os.path.exists(LIB_TGMS):
        build_tgms()
    return _lib.load()


@pytest.mark.parametrize("method", [0, 1, 2])
def test_plan_shards_matches_python_planner(lib, method):
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import plan_shards
    rng = np.random.default_rng(method)
    cases = [S.ragged_batch(int(rng.integers(1, 5000)), 1, 16, seed=int(s))[0] for s in rng.integers(0, 1 << 30, 12)]
    cases += [S.uniform_batch(1000, 10)[0], S.uniform_batch(7, 3)[0], np.array([0, 16], np.int32),
              S.ragged_batch(1048576 // 16, 2, 16)[0]]
    for so in cases:
        for parts in (1, 2, 3, 4, 5, 7, 8, 9, 16):
            got = plan_shards(so, parts, method)
            ref = SH.ragged_bounds(so, parts, method if method == 1 else 0)
            np.testing.assert_array_equal(got, ref.astype(np.int32))


def test_plan_shards_config5_share(lib):
    """The config-5 split used by bench.py and tests/test_gpu_configs.py."""
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import plan_shards
    so, _, _ = S.ragged_batch(1048576, 2, 16)
    got = plan_shards(so, 8)
    np.testing.assert_array_equal(got, SH.ragged_bounds(so, 8).astype(np.int32))
    sizes = np.diff(got)
    assert sizes.min() > 120000 and sizes.max() < 140000


def test_plan_shards_empty_and_invalid(lib):
    from trajectory_generator_ros2_amd import ERR_INVALID_ARG, TgmsError
    from trajectory_generator_ros2_amd.solver import plan_shards
    np.testing.assert_array_equal(plan_shards(np.zeros(1, np.int32), 4), np.zeros(5, np.int32))
    for so, parts in [(np.array([0, 2, 2], np.int32), 2), (np.array([1, 2], np.int32), 2),
                      (np.array([0, 3], np.int32), 0)]:
        with pytest.raises(TgmsError) as e:
            plan_shards(so, parts)
        assert e.value.status == ERR_INVALID_ARG


def test_create_multi_fails_loudly_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from trajectory_generator_ros2_amd import ERR_NO_DEVICE, TgmsError
    from trajectory_generator_ros2_amd.solver import Solver
    with pytest.raises(TgmsError) as ei:
        Solver(device_count=2)
    assert ei.value.status == ERR_NO_DEVICE


def test_rccl_is_loaded_not_linked(lib):
    from trajectory_generator_ros2_amd.build import LIB_TGMS
    deps = subprocess.run(["readelf", "-d", LIB_TGMS], capture_output=True, text=True, check=True).stdout
    assert "rccl" not in deps
    strings = open(LIB_TGMS, "rb").read()
    assert b"librccl.so.1" in strings and b"ncclCommInitAll" in strings


@pytest.mark.parametrize("method", [0, 1, 2])
def test_plan_shards_uniform_fast_path(lib, method):
    """Uniform batches take a closed-form path in the C planner (no per-trajectory
    prefix); it must cut exactly where the general rule and shard.ragged_bounds do."""
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd.solver import plan_shards
    for B, M in [(1048576, 10), (1048575, 10), (131072, 16), (999, 1), (5, 7), (1, 3), (3, 2)]:
        so = (np.arange(B + 1, dtype=np.int64) * M).astype(np.int32)
        for parts in (1, 2, 3, 4, 5, 7, 8, 13):
            got = plan_shards(so, parts, method)
            ref = SH.ragged_bounds(so, parts, method if method == 1 else 0)
            np.testing.assert_array_equal(got, ref.astype(np.int32), err_msg=f"B={B} M={M} parts={parts}")


@pytest.mark.parametrize("method", [0, 1])
def test_plan_shards_uniform_beyond_2_53(lib, method):
    """A uniform batch whose total cost passes 2^53 (the dense cost at a huge M): the
    running sum rounds in fp64, so the closed-form fast path would cut elsewhere; the
    planner then takes the general prefix-sum rule and still matches shard.ragged_bounds
    (ADVICE r03)."""
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd.solver import plan_shards
    M = 1 << 20
    so = (np.arange(1001, dtype=np.int64) * M).astype(np.int32)
    assert 1000 * float(14 * M + 2) ** 3 > 2.0 ** 53 or method == 0
    for parts in (2, 3, 7, 8):
        np.testing.assert_array_equal(plan_shards(so, parts, method), SH.ragged_bounds(so, parts, method).astype(np.int32))
