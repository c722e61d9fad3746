#!/bin/bash
# session g: config-5 class boundary / joint-axes variants, alternating, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c5var
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2; do
  for lib in default $V/libtgms_nojoint.so $V/libtgms_tw6.so $V/libtgms_tw8.so $V/libtgms_tw9.so $V/libtgms_tw10.so; do
    if [ $lib = default ]; then
      timeout -k 10 120 python3 scripts/c5bench.py >> $OUT/c5var.jsonl 2>> $OUT/c5var.err; c=$?
    else
      TGMS_LIB=$lib timeout -k 10 120 python3 scripts/c5bench.py >> $OUT/c5var.jsonl 2>> $OUT/c5var.err; c=$?
    fi
    echo "$lib exit $c"; [ $c -eq 0 ] || exit $c
  done
done
cat $OUT/c5var.jsonl
