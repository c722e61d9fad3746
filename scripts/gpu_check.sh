#!/bin/bash
# One GPU-box session: parity tests, headline bench, rocprofv3 kernel-trace summaries.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ok() { local c=$1; [ "$c" -eq 0 ] || [ "$c" -eq 1 ]; }   # 1 = test failure, keep going
SIDE_OFF="--dense-steps 0 --band-steps 0 --sample-traj 0 --config5 0 --config4 0 --cache-resident 0 --host-line 0 --node-line 0"

timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; c=$?
echo "pytest exit $c"; tail -5 $OUT/pytest_gpu.log
ok $c || exit $c

timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; c=$?
echo "bench exit $c"; cat $OUT/bench.json; tail -3 $OUT/bench.err
[ $c -eq 0 ] || exit $c

# the headline launch alone (its average duration must agree with the bench line's)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 $SIDE_OFF > $OUT/prof_bench.json 2> $OUT/prof.err; c=$?
echo "rocprof (headline) exit $c"
[ $c -eq 0 ] || exit $c
# every side line (dense KKT, sampler, config 4/5, cache-resident loop, host and node paths)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_full -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --dense-steps 2 > $OUT/prof_full_bench.json 2> $OUT/prof_full.err; c=$?
echo "rocprof (full) exit $c"
find $OUT/prof $OUT/prof_full -name '*stats*'
exit $c
