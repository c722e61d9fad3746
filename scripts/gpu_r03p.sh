#!/bin/bash
# session p: band-KKT quad kernel at one wavefront per SIMD (no scratch): band/edge/multi/
# capture tests, diagnosis at scale (persistent-grid reuse, M = 3/10/16), timing vs round 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py tests/test_gpu_multi.py tests/test_gpu_capture.py > $OUT/pytest_p.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_p.log
[ $c -eq 0 ] || exit $c
for c in "131072 16 7000" "131072 16 1" "40000 16 7000" "131072 10 7000" "20001 3 910" "262144 10 5"; do
  set -- $c
  KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 60 python3 scripts/band_diag.py >> $OUT/diag_p.jsonl 2>> $OUT/diag_p.err || exit 1
done
cut -c1-200 $OUT/diag_p.jsonl
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2; do
for lib in default $V/libtgms_oldband.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_p.jsonl 2>> $OUT/band_p.err || exit 1
done
done
cat $OUT/band_p.jsonl
