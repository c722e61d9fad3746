#!/bin/bash
# build a variant whose tgms_sample is compiled with extra flags
set -e
cd /root/repo
NAME=$1; shift
P=trajectory_generator_ros2_amd
mkdir -p $P/lib/variants $P/build/variants
OBJS=""
for f in tgms_reduced tgms_dense tgms_sample tgms_capi; do
  obj=$P/build/variants/${f}__$NAME.o; OBJS="$OBJS $obj"
  if [ "$f" = tgms_sample ]; then hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc "$@" -c $P/csrc/$f.hip -o $obj;
  else cp $P/build/$f.hip.o $obj; fi
done
hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libtgms_$NAME.so $OBJS
