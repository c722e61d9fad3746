#!/bin/bash
# session i: smoke, the whole -m gpu suite, bench (in-process full-size lines), bench with the
# N > 1 child-process path rehearsed on one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_i.log 2>&1; c=$?
echo "smoke exit $c"; tail -2 $OUT/smoke_i.log; [ $c -eq 0 ] || exit $c
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_i.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_i.log
[ $c -eq 0 ] || [ $c -eq 1 ] || exit $c
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 > $OUT/bench_i.json 2> $OUT/bench_i.err; c=$?
echo "bench exit $c"; [ $c -eq 0 ] || exit $c
TGMS_BENCH_FULL_CHILD=1 timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --dense-steps 0 --band-steps 0 --sample-traj 0 --host-line 0 --node-line 0 --cache-resident 0 > $OUT/bench_i_child.json 2> $OUT/bench_i_child.err; c=$?
echo "bench child exit $c"
exit $c
