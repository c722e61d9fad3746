#!/bin/bash
# round 4 session b: the round-3 quad kernel (192-B slab rows, 51c2b07) at two waves per SIMD
# (grids of 1, 2 and 3 workgroups per CU) at the shapes that failed in round 3; the
# refactored multi-GPU pipeline (host planner) through the multi / capture tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in q192w2 q192w2c8 q192w2c12 v2c8; do
  for c in "131072 16 7000" "131072 16 1" "40000 16 7000" "131072 10 7000" "20001 3 910"; do
    set -- $c
    echo "$lib $c $(TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_diag.py 2>> $OUT/diag_b.err | cut -c1-300)" >> $OUT/diag_b.txt || exit 1
  done
  echo "$lib done"
done
cat $OUT/diag_b.txt
for rep in 1 2 3; do
for lib in default $V/libtgms_v2c8.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_b.jsonl 2>> $OUT/band_b.err || exit 1
done
done
cut -c1-150 $OUT/band_b.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_capture.py tests/test_gpu_edges.py > $OUT/pytest_b.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_b.log
exit $c
