#!/bin/bash
# Copy the summaries of scripts/gpu_round.sh (gpurun_out/) into profiles/ (tracked).
set -eu
cd "$(dirname "$0")/.."
R=${1:-r01}
cp gpurun_out/bench.json profiles/${R}_bench.json
cp gpurun_out/prof_bench.json profiles/${R}_prof_bench.json
cp gpurun_out/prof/run_kernel_stats.csv profiles/${R}_kernel_stats.csv
cp gpurun_out/prof_full/run_kernel_stats.csv profiles/${R}_kernel_stats_full.csv
cp gpurun_out/prof_full_bench.json profiles/${R}_prof_full_bench.json
python3 scripts/pmc_traffic.py gpurun_out/pmc B65536_M10_reduced
T=$(mktemp -d); mkdir -p $T/rot
ln -s $PWD/gpurun_out/pmc/rot_FETCH_SIZE $T/rot/p1; ln -s $PWD/gpurun_out/pmc/rot_WRITE_SIZE $T/rot/p2
python3 scripts/pmc_traffic.py $T/rot B65536_M10_reduced_rotating
mkdir -p $T/sum; ln -s $PWD/gpurun_out/pmc $T/sum/reduced
python3 scripts/kpmc_summary.py $T/sum k_reduced_uniform > profiles/${R}_pmc_summary.txt
rm -rf $T
cat profiles/${R}_pmc_summary.txt
