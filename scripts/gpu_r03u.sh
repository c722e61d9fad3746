#!/bin/bash
# session u: band-KKT slab rows of 176 B (the two zero slots no longer stored): band/edge/
# multi/capture tests, scale diagnosis, timing against the round-2 kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py tests/test_gpu_multi.py tests/test_gpu_capture.py > $OUT/pytest_u.log 2>&1; c=$?
echo "pytest exit $c"; tail -1 $OUT/pytest_u.log
[ $c -eq 0 ] || exit $c
for c in "131072 16 7000" "40000 16 7000" "131072 10 7000" "20001 3 910" "262144 10 5" "65536 1 3"; do
  set -- $c
  KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 60 python3 scripts/band_diag.py > $OUT/d.json 2>> $OUT/diag_u.err || exit 1
  echo "$(cut -c1-100 $OUT/d.json)"
done
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
for lib in default $V/libtgms_oldband.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_u.jsonl 2>> $OUT/band_u.err || exit 1
done
done
cut -c1-140 $OUT/band_u.jsonl
