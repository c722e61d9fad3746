#!/bin/bash
# The N > 1 control flow of bench.py (process group, graph capture under it, barriers,
# max-over-ranks timing, the config-4 pipelined gather and its bit-exact check) with two
# ranks sharing the box's one GPU over gloo — RCCL refuses two ranks on one device.
# The 8-GPU RCCL run itself is the driver's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 --cpu-seconds 2 \
    --dense-steps 1 --band-steps 1 --sample-traj 512 > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err
c=$?
echo "rc=$c"
tail -c 1500 gpurun_out/bench_n2_gloo.json
exit $c
