#!/bin/bash
# round 4 session l: persistent lane kernel (one wave per SIMD looping over tiles) against the
# shipped one at the config-4 shard (131,072) and config 3 (65,536), fresh batches, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
  for b in 131072 262144 65536; do
    for lib in default $V/libtgms_lpersist.so; do
      if [ $lib = default ]; then L=""; else L=$lib; fi
      TGMS_LIB=$L KB_B=$b KB_ROT=3 KB_K=30 timeout -k 10 200 python3 scripts/kbench.py >> $OUT/lp_l.jsonl 2>> $OUT/lp_l.err || exit 1
    done
  done
done
cut -c1-200 $OUT/lp_l.jsonl
