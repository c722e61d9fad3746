"""bench.py's `--gpus N` contract, on CPU: under a launcher N must
equal WORLD_SIZE; without one, a single process drives N devices and refuses when
fewer are visible -- never a mislabeled line."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_resolve_topology_cases():
    from bench import resolve_topology
    assert resolve_topology(1, {}, 1) == ("process", 1, 0, 0)
    assert resolve_topology(8, {}, 8) == ("process", 8, 0, 0)
    assert resolve_topology(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}, 8) == ("ranks", 2, 1, 1)
    assert resolve_topology(1, {"WORLD_SIZE": "1"}, 1) == ("ranks", 1, 0, 0)
    with pytest.raises(SystemExit, match="only 1 HIP device"):
        resolve_topology(2, {}, 1)
    with pytest.raises(SystemExit, match="WORLD_SIZE=1"):
        resolve_topology(8, {"WORLD_SIZE": "1"}, 8)
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        resolve_topology(8, {"WORLD_SIZE": "4", "RANK": "0"}, 8)
    with pytest.raises(SystemExit, match=">= 1"):
        resolve_topology(0, {}, 8)


def test_bench_refuses_more_gpus_than_visible():
    """`python bench.py --gpus 2` on a machine with fewer devices exits non-zero with a
    message before touching a GPU (here: none visible)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 but only" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_refuses_streams_that_would_share_a_batch():
    """With --streams S the timed steps alternate over S streams and step k solves batch
    k % sets: unless S divides sets, two steps in flight at once could write one batch.
    bench.py refuses before touching a GPU."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--streams", "3", "--sets", "4",
                        "--steps", "1"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "must be a multiple of --streams 3" in r.stderr
    assert r.stdout.strip() == ""
