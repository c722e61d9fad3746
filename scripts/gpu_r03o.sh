#!/bin/bash
# session o: band-KKT quad kernel, aligned slab layout: band/edge/multi tests, diagnosis at
# several batch sizes (persistent-grid reuse), timing against the round-2 kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py tests/test_gpu_multi.py tests/test_gpu_capture.py > $OUT/pytest_o.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_o.log
[ $c -eq 0 ] || exit $c
for b in 20001 40000 100000 262144; do
  for m in 3 10 16; do
    KB_B=$b KB_M=$m timeout -k 10 60 python3 scripts/band_diag.py >> $OUT/diag_o.jsonl 2>> $OUT/diag_o.err || exit 1
  done
done
cat $OUT/diag_o.jsonl
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2; do
for lib in default $V/libtgms_oldband.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_o.jsonl 2>> $OUT/band_o.err || exit 1
done
done
cat $OUT/band_o.jsonl
