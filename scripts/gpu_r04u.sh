#!/bin/bash
# round 4 session u: bounds guard in the device-side grouping: every GPU test, smoke, config-5 timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_u.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_u.log
[ $c -eq 0 ] || exit $c
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_u.log 2>&1 || exit 1
tail -1 $OUT/smoke_u.log
for rep in 1 2 3; do
  timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_u.jsonl 2>> $OUT/c5_u.err || exit 1
done
cut -c1-200 $OUT/c5_u.jsonl
