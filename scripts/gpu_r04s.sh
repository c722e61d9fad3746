#!/bin/bash
# round 4 session s: config 5 at full size, every call timed alone (events + host time)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python3 scripts/c5full_probe.py > $OUT/c5full_s.json 2> $OUT/c5full_s.err || exit 1
cat $OUT/c5full_s.json
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/c5ftrace -o run -- python3 scripts/c5full_probe.py > $OUT/c5ftrace.json 2> $OUT/c5ftrace.err || exit 1
