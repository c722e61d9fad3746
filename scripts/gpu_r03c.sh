#!/bin/bash
# session c: full GPU suite after the host-path / refine-cost changes, config-4/5 timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_c.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_c.log
[ $c -eq 0 ] || [ $c -eq 1 ] || exit $c
timeout -k 10 300 python3 scripts/c4full.py > $OUT/c4full_c.json 2> $OUT/c4full_c.err; c=$?
echo "c4 exit $c"; cat $OUT/c4full_c.json; [ $c -eq 0 ] || exit $c
timeout -k 10 300 python3 scripts/c5bench.py > $OUT/c5bench_c.json 2> $OUT/c5bench_c.err; c=$?
echo "c5 exit $c"; cat $OUT/c5bench_c.json; [ $c -eq 0 ] || exit $c
timeout -k 10 300 python3 scripts/bandbench.py > $OUT/band_c.json 2> $OUT/band_c.err; c=$?
echo "band exit $c"; cat $OUT/band_c.json
exit $c
