#!/bin/bash
# config-5 side line (ragged + 10 refinement steps) for the default build and every variant
set -u
shopt -s nullglob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in default trajectory_generator_ros2_amd/lib/variants/*.so; do
  if [ $so = default ]; then unset TGMS_LIB; else export TGMS_LIB=$PWD/$so; fi
  for i in 1 2; do
    echo -n "$(basename $so) "
    timeout -k 10 120 python3 bench.py --steps 5 --dense-steps 0 --sample-traj 0 --config4 0 --rotating 0 --host-line 0 \
      --node-line 0 --cpu-seconds 0 2>/dev/null | python3 -c "import json,sys; print(json.load(sys.stdin)['config5']['ms_per_batch'])" || exit 1
  done
done
