#!/bin/bash
# round 4 session c: band-KKT reproduction of the round-3 two-wave failure (51c2b07 quad
# kernel, 192-B slab rows, at 1/2/3 workgroups per CU) and the current kernel at two waves
# per SIMD (8 waves per CU: timing + scale diagnosis); dense KKT two-column panel vs the
# round-3 kernel (bit equality, timing); GPU tests of the changed paths
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in q192w2 q192w2c8 q192w2c12 v2c8; do
  for c in "131072 16 7000" "131072 16 1" "40000 16 7000" "131072 10 7000" "20001 3 910"; do
    set -- $c
    echo "$lib $c $(TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_diag.py 2>> $OUT/diag_c.err | cut -c1-300)" >> $OUT/diag_c.txt || exit 1
  done
  echo "$lib done"
done
cut -c1-200 $OUT/diag_c.txt
for rep in 1 2 3; do
for lib in default $V/libtgms_v2c8.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_c.jsonl 2>> $OUT/band_c.err || exit 1
done
done
cut -c1-150 $OUT/band_c.jsonl
TGMS_LIB=$V/libtgms_dense_panel.so KB_TAG=panel KB_MS=3,5,10 timeout -k 10 200 python3 scripts/dense_ab.py > $OUT/dense_c.jsonl 2>> $OUT/dense_c.err || exit 1
KB_TAG=old KB_MS=3,5,10 timeout -k 10 200 python3 scripts/dense_ab.py >> $OUT/dense_c.jsonl 2>> $OUT/dense_c.err || exit 1
KB_CMP=panel,old python3 scripts/dense_ab.py >> $OUT/dense_c.jsonl
rm -f $OUT/dense_*.npy
cat $OUT/dense_c.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_capture.py tests/test_gpu_edges.py tests/test_gpu_parity.py > $OUT/pytest_c.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_c.log
[ $c -eq 0 ] || exit $c
TGMS_LIB=$V/libtgms_dense_panel.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_multi.py -k "dense or goldens or method" > $OUT/pytest_c2.log 2>&1; c=$?
echo "pytest (dense panel) exit $c"; tail -3 $OUT/pytest_c2.log
exit $c
