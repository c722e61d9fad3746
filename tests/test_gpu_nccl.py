"""shard.pipelined_gather and ShardedBatch.gather on the nccl (RCCL) backend, world
size 1, in a fresh spawned process whose process group is created before any GPU
call (as bench.py creates it).  The N > 1 paths are covered with gloo on CPU
(tests/test_shard.py); an 8-GPU run is the driver's."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_pipelined_gather_nccl_world1():
    env = dict(os.environ)
    env.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()), "RANK": "0", "WORLD_SIZE": "1",
                "LOCAL_RANK": "0"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nccl_child.py")
    r = subprocess.run([sys.executable, "-u", child], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "NCCL_OK" in r.stdout
