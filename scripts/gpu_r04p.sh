#!/bin/bash
# round 4 session p: config-5 loop with a lane-per-trajectory class (M <= 10, default; lane7:
# M <= 7; nolane: the lane-pair classes only): GPU tests, agreement with the lane-pair loop,
# timing alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_p.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_p.log
[ $c -eq 0 ] || exit $c
timeout -k 10 120 python3 scripts/c5_equiv.py $OUT/c5_lane.npz || exit 1
TGMS_LIB=$V/libtgms_nolane.so timeout -k 10 120 python3 scripts/c5_equiv.py $OUT/c5_pair.npz || exit 1
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/c5_lane.npz"); b = np.load("gpurun_out/c5_pair.npz")
for k in a.files:
    x, y = a[k], b[k]
    if k.endswith("_st"):
        print(k, "equal", bool(np.array_equal(x, y)))
    else:
        ok = np.isfinite(y) & (y != 0)
        d = np.abs(x - y)
        print(k, "bit-equal", bool(np.array_equal(x, y, equal_nan=True)), "max rel", float((d[ok] / np.abs(y[ok])).max()) if ok.any() else 0.0,
              "zeros agree", bool(((x == 0) == (y == 0)).all()))
PY
rm -f $OUT/c5_lane.npz $OUT/c5_pair.npz
for rep in 1 2 3; do
  for lib in default $V/libtgms_nolane.so $V/libtgms_lane7.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_p.jsonl 2>> $OUT/c5_p.err || exit 1
  done
done
cut -c1-200 $OUT/c5_p.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5trace_p -o run -- python3 scripts/c5bench.py > $OUT/c5trace_p.json 2> $OUT/c5trace_p.err || exit 1
