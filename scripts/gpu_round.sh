#!/bin/bash
# parity + bench + kernel-trace + PMC in one box session
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh; c=$?
[ $c -eq 0 ] || [ $c -eq 1 ] || exit $c
bash scripts/gpu_profile.sh
