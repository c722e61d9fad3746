#!/bin/bash
# kbench.py over batch sizes (in and beyond the 256 MB Infinity Cache) for the default
# build and every variant under lib/variants
set -u
shopt -s nullglob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bsweep
for B in ${BS:-65536 131072 262144 524288}; do
  for so in default trajectory_generator_ros2_amd/lib/variants/*.so; do
    n=$(basename $so .so)
    if [ $so = default ]; then unset TGMS_LIB; else export TGMS_LIB=$PWD/$so; fi
    KB_B=$B timeout -k 10 120 python3 scripts/kbench.py > gpurun_out/bsweep/${n}_$B.json 2>gpurun_out/bsweep/${n}_$B.err; c=$?
    cat gpurun_out/bsweep/${n}_$B.json; [ $c -eq 0 ] || exit $c
    KB_ROT=4 KB_B=$B timeout -k 10 120 python3 scripts/kbench.py > gpurun_out/bsweep/${n}_${B}_rot.json 2>gpurun_out/bsweep/${n}_${B}_rot.err; c=$?
    cat gpurun_out/bsweep/${n}_${B}_rot.json; [ $c -eq 0 ] || exit $c
  done
done
