#!/bin/bash
# headline (kbench) and band (bandbench) timings for the default build and every variant
set -u
shopt -s nullglob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in default trajectory_generator_ros2_amd/lib/variants/*.so; do
  if [ $so = default ]; then unset TGMS_LIB; else export TGMS_LIB=$PWD/$so; fi
  timeout -k 10 120 python3 scripts/kbench.py || exit $?
  timeout -k 10 120 python3 scripts/bandbench.py || exit $?
done
