#!/bin/bash
# round 4 session r: chunked host validation, device-side M grouping in the refinement loop: every GPU test,
# config-5 timing, the full bench line (config5_full exposes the host planning)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_r.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_r.log
[ $c -eq 0 ] || exit $c
for rep in 1 2 3; do
  timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_r.jsonl 2>> $OUT/c5_r.err || exit 1
done
cut -c1-220 $OUT/c5_r.jsonl
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_r.json 2> $OUT/bench_r.err; c=$?
echo "bench exit $c"; tail -c 600 $OUT/bench_r.json
[ $c -eq 0 ] || exit $c
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5trace_r -o run -- python3 scripts/c5bench.py > $OUT/c5trace_r.json 2> $OUT/c5trace_r.err || exit 1
