#!/bin/bash
# build_variant.sh NAME [hipcc -D flags...] -> trajectory_generator_ros2_amd/lib/variants/libtgms_NAME.so
# VARIANT_FILES (default: every HIP source) names the sources compiled with the flags; the
# others are linked from the default build's objects (trajectory_generator_ros2_amd/build).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
P=trajectory_generator_ros2_amd
FILES=${VARIANT_FILES:-"tgms_reduced tgms_dense tgms_band tgms_sample tgms_capi"}
mkdir -p $P/lib/variants $P/build/variants
OBJS="$P/build/tgms_plan.cpp.o"
for f in tgms_reduced tgms_dense tgms_band tgms_sample tgms_capi; do
  src=$P/csrc/$f.hip
  if [[ " $FILES " == *" $f "* ]]; then
    obj=$P/build/variants/${f}__$NAME.o
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc "$@" -c $src -o $obj &
  else
    obj=$P/build/$f.hip.o
  fi
  OBJS="$OBJS $obj"
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libtgms_$NAME.so $OBJS -ldl
echo $P/lib/variants/libtgms_$NAME.so
