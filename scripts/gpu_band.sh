#!/bin/bash
# band-KKT: parity tests, then kernel timing of the default build and every variant
set -u
shopt -s nullglob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 120 --timeout-method thread > gpurun_out/band_test.log 2>&1; c=$?
tail -3 gpurun_out/band_test.log
[ $c -eq 0 ] || exit $c
for so in default trajectory_generator_ros2_amd/lib/variants/*.so; do
  if [ $so = default ]; then unset TGMS_LIB; else export TGMS_LIB=$PWD/$so; fi
  timeout -k 10 120 python3 scripts/bandbench.py || exit $?
done
