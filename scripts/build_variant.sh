#!/bin/bash
# build_variant.sh NAME [hipcc -D flags...] -> trajectory_generator_ros2_amd/lib/variants/libtgms_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
P=trajectory_generator_ros2_amd
mkdir -p $P/lib/variants $P/build/variants
OBJS=""
for f in tgms_reduced tgms_dense tgms_band tgms_sample tgms_capi; do
  src=$P/csrc/$f.hip; obj=$P/build/variants/${f}__$NAME.o
  OBJS="$OBJS $obj"
  if [ "$f" != tgms_sample ]; then  # the C ABI too: it shares compile-time knobs (class boundary)
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc "$@" -c $src -o $obj &
  else
    [ -f $P/build/$f.hip.o ] && cp $P/build/$f.hip.o $obj || hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$P/csrc -c $src -o $obj &
  fi
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libtgms_$NAME.so $OBJS
echo $P/lib/variants/libtgms_$NAME.so
