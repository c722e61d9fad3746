#!/bin/bash
# Copy the summaries of scripts/gpu_round.sh (gpurun_out/) into profiles/ (tracked):
# the bench lines, the rocprofv3 kernel-trace statistics of the headline-only and the
# full bench, and the PMC passes folded into profiles/pmc_traffic.json.
set -eu
cd "$(dirname "$0")/.."
R=${1:-r02}
cp gpurun_out/bench.json profiles/${R}_bench.json
cp gpurun_out/prof_bench.json profiles/${R}_prof_bench.json
cp gpurun_out/prof/run_kernel_stats.csv profiles/${R}_kernel_stats.csv
cp gpurun_out/prof_full/run_kernel_stats.csv profiles/${R}_kernel_stats_full.csv
cp gpurun_out/prof_full_bench.json profiles/${R}_prof_full_bench.json
if [ -d gpurun_out/pmc ]; then
  python3 scripts/pmc_traffic.py gpurun_out/pmc B65536_M10_reduced_sets4
  python3 - "$R" <<'PY'
import json, sys
d = json.load(open("profiles/pmc_traffic.json"))["B65536_M10_reduced_sets4"]
with open(f"profiles/{sys.argv[1]}_pmc_summary.txt", "w") as f:
    f.write(f"{d['kernel']}, headline bench (fresh batch every launch), mean per dispatch\n")
    f.write(f"HBM bytes/launch (FETCH_SIZE x2 + WRITE_SIZE): {d['hbm_bytes_per_launch']:.0f}\n")
    for k, v in sorted(d["other_counters"].items()):
        f.write(f"{k:28s} {v:16.1f}\n")
PY
  cat profiles/${R}_pmc_summary.txt
fi
