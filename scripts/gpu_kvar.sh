#!/bin/bash
# Kernel A/B: the default build against variant builds (scripts/build_variant.sh),
# config 3 re-solving one batch (rot 1) and rotating over 4 fresh batches (rot 4).
# usage: gpu_kvar.sh [variant names...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/kv.jsonl
for lib in default "$@"; do
  if [ $lib = default ]; then unset TGMS_LIB; else export TGMS_LIB=$PWD/trajectory_generator_ros2_amd/lib/variants/libtgms_$lib.so; fi
  for rot in 1 4; do
    KB_ROT=$rot timeout -k 10 120 python scripts/kbench.py >> gpurun_out/kv.jsonl 2>>gpurun_out/kv.err || exit $?
  done
done
cat gpurun_out/kv.jsonl
