#!/bin/bash
# One GPU-box session: parity tests, headline bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ok() { local c=$1; [ "$c" -eq 0 ] || [ "$c" -eq 1 ]; }   # 1 = test failure, keep going

timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; c=$?
echo "pytest exit $c"; tail -5 $OUT/pytest_gpu.log
ok $c || exit $c

timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; c=$?
echo "bench exit $c"; cat $OUT/bench.json; tail -3 $OUT/bench.err
[ $c -eq 0 ] || exit $c

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --dense-steps 2 > $OUT/prof_bench.json 2> $OUT/prof.err; c=$?
echo "rocprof exit $c"
find $OUT/prof -name '*stats*' | head
exit $c
