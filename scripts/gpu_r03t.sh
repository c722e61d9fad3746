#!/bin/bash
# session t: band-KKT step latency variants (no per-step scheduling barrier, pairwise
# pivot-search trees, both) against the shipped build, config 3, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
for lib in default $V/libtgms_nosb.so $V/libtgms_tree.so $V/libtgms_both.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_t.jsonl 2>> $OUT/band_t.err || exit 1
done
done
cut -c1-200 $OUT/band_t.jsonl
