#!/bin/bash
# round 4 end-of-round session: smoke, every GPU test, headline bench, kernel-trace summaries
# (headline alone and every side line), headline PMC traffic passes (folded into
# gpurun_out/pmc_traffic.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; c=$?
echo "smoke exit $c"; tail -1 $OUT/smoke.log
[ $c -eq 0 ] || exit $c
bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_profile.sh || exit $?
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
