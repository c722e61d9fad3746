#!/bin/bash
# build_variant_all.sh NAME [hipcc -D flags...]: every HIP source with the flags -> lib/variants/libtgms_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
P=trajectory_generator_ros2_amd
mkdir -p $P/lib/variants $P/build/variants
OBJS=""
for f in tgms_reduced tgms_dense tgms_sample tgms_capi; do
  obj=$P/build/variants/${f}__$NAME.o; OBJS="$OBJS $obj"
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc "$@" -c $P/csrc/$f.hip -o $obj &
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libtgms_$NAME.so $OBJS
echo $P/lib/variants/libtgms_$NAME.so
