#!/bin/bash
# round 4 session v: lane-pair forward substitution reading the next knot's LDS values one
# step ahead (pf2: forward and back substitution) against the shipped build: config-5 timing alternating, parity tests on pf
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
  for lib in default $V/libtgms_pf2.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_v.jsonl 2>> $OUT/c5_v.err || exit 1
  done
done
cut -c1-200 $OUT/c5_v.jsonl
for m in 3 5 13; do
  for lib in default $V/libtgms_pf2.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L KB_M=$m KB_ROT=3 KB_K=20 timeout -k 10 300 python3 scripts/kbench.py >> $OUT/pair_v.jsonl 2>> $OUT/pair_v.err || exit 1
  done
done
cut -c1-160 $OUT/pair_v.jsonl
TGMS_LIB=$V/libtgms_pf2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_full_configs.py > $OUT/pytest_v.log 2>&1; c=$?
echo "pytest pf2 exit $c"; tail -2 $OUT/pytest_v.log
exit $c
