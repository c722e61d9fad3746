#!/bin/bash
# session n: band-KKT slab layout (64-B runs) + one-wave-per-SIMD variant + forward-only ablation
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py > $OUT/pytest_n.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_n.log
[ $c -eq 0 ] || exit $c
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2; do
for lib in default $V/libtgms_wpe1.so $V/libtgms_noback.so $V/libtgms_oldband.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_n.jsonl 2>> $OUT/band_n.err || exit 1
done
done
cat $OUT/band_n.jsonl
