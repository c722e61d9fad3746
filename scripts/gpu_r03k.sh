#!/bin/bash
# session k: quad band-KKT kernel (8-lane slot-order back substitution): parity, then timing against the round-2 row-lane kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py > $OUT/pytest_l.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_l.log
[ $c -eq 0 ] || exit $c
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_l.jsonl 2>> $OUT/band_l.err || exit 1
  TGMS_LIB=trajectory_generator_ros2_amd/lib/variants/libtgms_oldband.so timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_l.jsonl 2>> $OUT/band_l.err || exit 1
done
cat $OUT/band_l.jsonl
