#!/bin/bash
# round-3 first box session: occupancy store probe, the new GPU tests, bench with the full-size lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./scripts/micro/occstore > $OUT/occstore.txt 2>&1; c=$?
echo "occstore exit $c"; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_capture.py tests/test_gpu_edges.py tests/test_gpu_full_configs.py > $OUT/pytest_new.log 2>&1; c=$?
echo "pytest exit $c"; tail -5 $OUT/pytest_new.log
[ $c -eq 0 ] || [ $c -eq 1 ] || exit $c
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --dense-steps 0 > $OUT/bench_r03a.json 2> $OUT/bench_r03a.err; c=$?
echo "bench exit $c"; tail -3 $OUT/bench_r03a.err
exit $c
