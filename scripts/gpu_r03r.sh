#!/bin/bash
# session r: band KKT as two kernels (forward elimination / back substitution) with the
# chunk pipeline on two streams: band/edge/multi/capture tests, scale diagnosis, timing of
# the shipped build (forward one wave per SIMD beside the back substitution), the two-wave
# forward variant and the round-2 kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py tests/test_gpu_multi.py tests/test_gpu_capture.py > $OUT/pytest_r.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_r.log
[ $c -eq 0 ] || exit $c
V=trajectory_generator_ros2_amd/lib/variants
for lib in default; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  for c in "131072 16 7000" "40000 16 7000" "131072 10 7000" "20001 3 910" "262144 10 5"; do
    set -- $c
    TGMS_LIB=$L KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 60 python3 scripts/band_diag.py >> $OUT/diag_r.jsonl 2>> $OUT/diag_r.err || exit 1
  done
done
cut -c1-120 $OUT/diag_r.jsonl
for rep in 1 2; do
for lib in default $V/libtgms_oldband.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_r.jsonl 2>> $OUT/band_r.err || exit 1
done
done
cat $OUT/band_r.jsonl
