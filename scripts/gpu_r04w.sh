#!/bin/bash
# round 4 session w: the joint-axes lane-pair solve (one-wave class, M >= 14) with the LDS
# values read one step ahead (jpf) against the shipped build: config-5 timing alternating,
# uniform M = 14/16, parity tests on jpf
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
  for lib in default $V/libtgms_jpf.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_w.jsonl 2>> $OUT/c5_w.err || exit 1
  done
done
cut -c1-200 $OUT/c5_w.jsonl
for m in 14 16; do
  for lib in default $V/libtgms_jpf.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L KB_M=$m KB_ROT=3 KB_K=20 timeout -k 10 300 python3 scripts/kbench.py >> $OUT/joint_w.jsonl 2>> $OUT/joint_w.err || exit 1
  done
done
cut -c1-160 $OUT/joint_w.jsonl
TGMS_LIB=$V/libtgms_jpf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_full_configs.py > $OUT/pytest_w.log 2>&1; c=$?
echo "pytest jpf exit $c"; tail -2 $OUT/pytest_w.log
exit $c
