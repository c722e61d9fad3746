#!/bin/bash
# session s: split band kernels, chunk pipeline on / off (TGMS_BAND_NOPIPE): scale diagnosis
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for np in 0 1; do
  for c in "131072 16 7000" "131072 10 7000" "65536 10 3"; do
    set -- $c
    if [ $np = 1 ]; then export TGMS_BAND_NOPIPE=1; else unset TGMS_BAND_NOPIPE; fi
    KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 60 python3 scripts/band_diag.py > $OUT/d.json 2>> $OUT/diag_s.err || exit 1
    echo "nopipe=$np $(cut -c1-160 $OUT/d.json)"
  done
done
unset TGMS_BAND_NOPIPE
timeout -k 10 60 python3 scripts/bandbench.py && TGMS_BAND_NOPIPE=1 timeout -k 10 60 python3 scripts/bandbench.py
