#!/bin/bash
# round 4 session t: one-device multi handle -> single-device refinement loop (graph,
# device grouping): every GPU test, the full-size probe, the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_t.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_t.log
[ $c -eq 0 ] || exit $c
timeout -k 10 200 python3 scripts/c5full_probe.py > $OUT/c5full_t.json 2> $OUT/c5full_t.err || exit 1
cat $OUT/c5full_t.json
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_t.json 2> $OUT/bench_t.err; c=$?
echo "bench exit $c"
exit $c
