#!/bin/bash
# round 4 session d: band KKT with the quad back substitution (one pass of 16 trajectories,
# each lane reading back its own slab slots) at one and two waves per SIMD: timing against
# the shipped kernel and the two-wave build, scale diagnosis, band GPU tests on the variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
for lib in default $V/libtgms_b4.so $V/libtgms_b4w2.so $V/libtgms_v2c8.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_d.jsonl 2>> $OUT/band_d.err || exit 1
done
done
cut -c1-150 $OUT/band_d.jsonl
for lib in b4 b4w2; do
  for c in "131072 16 7000" "131072 16 1" "40000 16 7000" "131072 10 7000" "20001 3 910" "65536 1 3"; do
    set -- $c
    echo "$lib $c $(TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_diag.py 2>> $OUT/diag_d.err | cut -c1-120)" >> $OUT/diag_d.txt || exit 1
  done
done
cat $OUT/diag_d.txt
for lib in b4 b4w2; do
  TGMS_LIB=$V/libtgms_$lib.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py tests/test_gpu_capture.py tests/test_gpu_multi.py -k "band or method" > $OUT/pytest_d_$lib.log 2>&1; c=$?
  echo "pytest $lib exit $c"; tail -2 $OUT/pytest_d_$lib.log
  [ $c -eq 0 ] || exit $c
done
# uniform M = 12/14/16: the lane kernel (spills to scratch at these M) against the lane-pair
# kernel (TGMS_LANE_MAX_M=10 variant), fresh batches
for m in 12 14 16; do
  for lib in default $V/libtgms_lanemax10.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L KB_M=$m KB_ROT=3 KB_K=20 timeout -k 10 300 python3 scripts/kbench.py >> $OUT/lane_d.jsonl 2>> $OUT/lane_d.err || exit 1
  done
done
cut -c1-200 $OUT/lane_d.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_parity.py > $OUT/pytest_d_main.log 2>&1; c=$?
echo "pytest main exit $c"; tail -2 $OUT/pytest_d_main.log
exit $c
