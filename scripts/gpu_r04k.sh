#!/bin/bash
# round 4 session k: config-5 class boundary with the merged last pass (default 11 / 13 /
# 15), alternating; a kernel + memory-copy trace of the default build's calls
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
  for lib in default $V/libtgms_tw13.so $V/libtgms_tw15.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_k.jsonl 2>> $OUT/c5_k.err || exit 1
  done
done
cut -c1-220 $OUT/c5_k.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/c5trace -o run -- python3 scripts/c5bench.py > $OUT/c5trace.json 2> $OUT/c5trace.err || exit 1
find $OUT/c5trace -name '*.csv'
