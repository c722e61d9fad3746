#!/bin/bash
# sampler micro-benchmark for the default build and every variant under lib/variants
set -u
shopt -s nullglob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for N in ${SB_NS:-4096 1024}; do
  for so in default trajectory_generator_ros2_amd/lib/variants/*.so; do
    if [ $so = default ]; then unset TGMS_LIB; else export TGMS_LIB=$PWD/$so; fi
    echo "== $(basename $so) N=$N"
    SB_N=$N timeout -k 10 120 python3 scripts/sbench.py || exit $?
  done
done
