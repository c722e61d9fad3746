#!/bin/bash
# round 4 session g: (1) reproduction of round 3's two-wave band failure with that round's
# kernel (51c2b07: 192-B slab rows) at one and two waves per SIMD, and the current kernel at
# two waves per SIMD on the same one-workgroup-per-CU grid (HW_ID status words); (2) timing:
# shipped / quad back substitution (b4, one and two waves) / current kernel at two waves per
# SIMD on a two-workgroups-per-CU grid; (3) band GPU tests on the variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in q192w1h q192w2h v2h4; do
  for c in "131072 16 7000" "40000 16 7000" "131072 10 7000" "40000 3 910" "20001 3 910"; do
    set -- $c
    echo "== $lib $c" >> $OUT/hwdiag_g.jsonl
    TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_hwdiag.py >> $OUT/hwdiag_g.jsonl 2>> $OUT/hwdiag_g.err || exit 1
  done
  echo "$lib done"
done
python3 - <<'PY'
import json
for l in open("gpurun_out/hwdiag_g.jsonl"):
    if l.startswith("=="): print(l.strip()); continue
    d = json.loads(l); print(" rep", d["rep"], "n_bad", d["n_bad"], "max_err", "%.2e" % d["max_err"], "slots", d["slots"], "tg_bad", d["tg"]["bad"][:4], "wave_bad", d["wave"]["bad"][:4], "simd_bad", d["simd"]["bad"], "tg_all", d["tg"]["all"][:4], "cus_2tg", d["cus_with_2plus_tg"])
PY
for rep in 1 2 3; do
for lib in default $V/libtgms_b4.so $V/libtgms_b4w2.so $V/libtgms_v2c8.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_g.jsonl 2>> $OUT/band_g.err || exit 1
done
done
cut -c1-160 $OUT/band_g.jsonl
for lib in b4 b4w2 v2c8; do
  TGMS_LIB=$V/libtgms_$lib.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py tests/test_gpu_edges.py tests/test_gpu_capture.py tests/test_gpu_multi.py -k "band or method or breakdown" > $OUT/pytest_g_$lib.log 2>&1; c=$?
  echo "pytest $lib exit $c"; tail -2 $OUT/pytest_g_$lib.log
  [ $c -eq 0 ] || exit $c
done
