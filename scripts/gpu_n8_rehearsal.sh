#!/bin/bash
# bench.py's N = 8 control flow (8-way cost-balanced config-5 shards, the config-4 gather
# of 8 pieces, max/min over 8 ranks) with eight ranks sharing the box's one GPU over gloo.
# Timings are meaningless (eight processes on one device); the run checks the code path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 8 --backend gloo --steps 5 --warmup 2 --cpu-seconds 2 \
    --dense-steps 1 --band-steps 1 --sample-traj 512 > gpurun_out/bench_n8_gloo.json 2> gpurun_out/bench_n8_gloo.err
c=$?
echo "rc=$c"
tail -c 2500 gpurun_out/bench_n8_gloo.json
exit $c
