#!/bin/bash
# round 4 session e (first of the re-entered session): every GPU test (with the new band
# regression shapes), smoke, headline bench, kernel-trace summaries
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; c=$?
echo "smoke exit $c"; tail -2 $OUT/smoke.log
[ $c -eq 0 ] || exit $c
bash scripts/gpu_check.sh
