#!/bin/bash
# session h: config-5 launch variants (graph vs direct launches, class order), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c5var
mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 120 python3 scripts/c5bench.py >> $OUT/c5launch.jsonl 2>> $OUT/c5launch.err || exit 1
  TGMS_NO_GRAPH=1 timeout -k 10 120 python3 scripts/c5bench.py | sed 's/"lib"/"variant": "no_graph", "lib"/' >> $OUT/c5launch.jsonl 2>> $OUT/c5launch.err || exit 1
  TGMS_LOOP_CLASS_A_FIRST=1 timeout -k 10 120 python3 scripts/c5bench.py | sed 's/"lib"/"variant": "a_first", "lib"/' >> $OUT/c5launch.jsonl 2>> $OUT/c5launch.err || exit 1
  TGMS_NO_GRAPH=1 TGMS_LOOP_CLASS_A_FIRST=1 timeout -k 10 120 python3 scripts/c5bench.py | sed 's/"lib"/"variant": "no_graph_a_first", "lib"/' >> $OUT/c5launch.jsonl 2>> $OUT/c5launch.err || exit 1
done
cat $OUT/c5launch.jsonl
