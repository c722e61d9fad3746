#!/bin/bash
# time every variant library under lib/variants (plus the default build) with kbench.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/kbench.py > gpurun_out/kb_default.json 2>gpurun_out/kb_default.err; c=$?
cat gpurun_out/kb_default.json; [ $c -eq 0 ] || exit $c
for so in trajectory_generator_ros2_amd/lib/variants/*.so; do
  n=$(basename $so .so)
  TGMS_LIB=$PWD/$so timeout -k 10 120 python3 scripts/kbench.py > gpurun_out/kb_$n.json 2>gpurun_out/kb_$n.err; c=$?
  cat gpurun_out/kb_$n.json; [ $c -eq 0 ] || exit $c
done
