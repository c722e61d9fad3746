"""Child process of tests/test_gpu_nccl.py (not collected by pytest): one rank of a
world-size-1 nccl (RCCL) process group, started before this process makes any GPU
call, runs shard.pipelined_gather and ShardedBatch.gather through RCCL and checks
them against the unsharded solve.  Prints NCCL_OK on success."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from trajectory_generator_ros2_amd import shard as SH
    from trajectory_generator_ros2_amd import synthetic as S
    from trajectory_generator_ros2_amd.solver import Solver

    B, M = 8192, 10
    _, W, T = S.uniform_batch(B, M, seed=31)
    dW, dT = torch.from_numpy(W).cuda(), torch.from_numpy(T).cuda()
    with Solver(0) as s:
        ref = torch.empty((B, M, 3, 8), dtype=torch.float64, device="cuda")
        s.solve_uniform_device(B, M, dW, dT, ref)
        dC = torch.full_like(ref, float("nan"))
        out = torch.full((1, B, M, 3, 8), float("nan"), dtype=torch.float64, device="cuda")
        sp = torch.cuda.current_stream().cuda_stream
        works = SH.pipelined_gather(lambda lo, hi: s.solve_uniform_device(hi - lo, M, dW[lo:hi], dT[lo:hi],
                                                                          dC[lo:hi], stream=sp),
                                    dC, 4, dst=0, out=out)
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        assert torch.equal(out[0], ref), "pipelined_gather over RCCL differs from the unsharded solve"
        # ShardedBatch.gather of a ragged batch through the same communicator
        so, Wr, Tr = S.ragged_batch(3000, 2, 16, seed=32)
        sb = SH.ShardedBatch(so, Wr, Tr, rank=0, world=1)
        C, st = sb.solve(lambda a, b, c, d: s.solve(a, b, c, d)[:2])
        got = sb.gather(torch.from_numpy(C).cuda(), torch.from_numpy(st).cuda(), dst=0)
        assert got is not None and np.array_equal(got[0].cpu().numpy(), C)
    dist.destroy_process_group()
    print("NCCL_OK", flush=True)


if __name__ == "__main__":
    main()
