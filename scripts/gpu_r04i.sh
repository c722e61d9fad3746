#!/bin/bash
# round 4 session i: (1) round 3's committed two-wave band kernel built exactly as then (no
# HW_ID patch) on grids of two and three workgroups per CU, three runs per shape;
# (2) config 5: the fused loop's last pass emitting the coefficients and the cost from one
# solve (default) against the previous build (c5old): equality and timing; GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in q192w2c8 q192w2c12; do
  for c in "131072 16 7000" "131072 16 1" "40000 16 7000" "131072 10 7000" "40000 3 910" "20001 3 910"; do
    set -- $c
    for rep in 1 2 3; do
      echo "$lib $c $(TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_diag.py 2>> $OUT/diag_i.err | cut -c1-200)" >> $OUT/diag_i.txt || exit 1
    done
  done
done
cut -c1-120 $OUT/diag_i.txt
timeout -k 10 120 python3 scripts/c5_equiv.py $OUT/c5_new.npz || exit 1
TGMS_LIB=$V/libtgms_c5old.so timeout -k 10 120 python3 scripts/c5_equiv.py $OUT/c5_old.npz || exit 1
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/c5_new.npz"); b = np.load("gpurun_out/c5_old.npz")
for k in a.files:
    x, y = a[k], b[k]
    if k.endswith("_cost"):
        ok = np.isfinite(y)
        print(k, "bit-equal", bool((x == y).all()), "max rel", float((np.abs(x - y)[ok] / np.abs(y[ok])).max()))
    else:
        print(k, "bit-equal", bool(np.array_equal(x, y, equal_nan=True)))
PY
rm -f $OUT/c5_new.npz $OUT/c5_old.npz
for rep in 1 2 3; do
  for lib in default $V/libtgms_c5old.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_i.jsonl 2>> $OUT/c5_i.err || exit 1
  done
done
cut -c1-200 $OUT/c5_i.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_full_configs.py tests/test_gpu_multi.py tests/test_gpu_capture.py tests/test_gpu_edges.py tests/test_gpu_parity.py > $OUT/pytest_i.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_i.log
exit $c
