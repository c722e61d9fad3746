#!/bin/bash
# round 4 session a: band-KKT wrong-result diagnosis.  HW_ID-instrumented builds (status word =
# where each trajectory ran): one wave per SIMD (shipped), two waves per SIMD (spilling), two
# waves + full agent fences at the slab hand-off, two waves on a grid of two workgroups per CU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in v1h v2h v2hf v2h8; do
  for c in "131072 16 7000" "40000 16 7000" "131072 10 7000" "20001 3 910"; do
    set -- $c
    echo "== $lib $c" >> $OUT/hwdiag_a.jsonl
    TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_hwdiag.py >> $OUT/hwdiag_a.jsonl 2>> $OUT/hwdiag_a.err || exit 1
  done
  echo "$lib done"
done
for lib in default $V/libtgms_v2.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_a.jsonl 2>> $OUT/band_a.err || exit 1
done
cat $OUT/band_a.jsonl
