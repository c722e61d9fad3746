#!/bin/bash
# round 4 session j: the two-wave band build as the default: every GPU test, smoke, bench,
# band PMC passes (summary), kernel-trace summaries
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; c=$?
echo "smoke exit $c"; tail -1 $OUT/smoke.log
[ $c -eq 0 ] || exit $c
bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_bandpmc.sh || exit $?
python3 scripts/band_pmc_summary.py gpurun_out/bandpmc "round 4: quad mapping, two wavefronts per SIMD (two workgroups per CU), 176-B slab rows" > $OUT/band_summary.txt
cat $OUT/band_summary.txt
