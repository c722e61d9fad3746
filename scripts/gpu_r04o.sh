#!/bin/bash
# round 4 session o: lane kernel up to M = 12 (M = 14, 16 on the lane pair): every GPU test,
# uniform M = 14/16 timing; config-5 kernel + memory-copy trace with the class boundary at 13
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_o.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_o.log
[ $c -eq 0 ] || exit $c
for m in 14 16; do
  KB_M=$m KB_ROT=3 KB_K=20 timeout -k 10 300 python3 scripts/kbench.py >> $OUT/lane_o.jsonl 2>> $OUT/lane_o.err || exit 1
done
cut -c1-200 $OUT/lane_o.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/c5trace_o -o run -- python3 scripts/c5bench.py > $OUT/c5trace_o.json 2> $OUT/c5trace_o.err || exit 1
cat $OUT/c5trace_o.json
