#!/bin/bash
# session e: refine-loop times in registers (8 waves/CU for the M<=11 class): parity + timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_full_configs.py > $OUT/pytest_e.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_e.log
[ $c -eq 0 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5prof_e -o run --output-format csv -- python3 scripts/c5bench.py > $OUT/c5prof_e.json 2> $OUT/c5prof_e.err; c=$?
echo "c5prof exit $c"; cat $OUT/c5prof_e.json; grep refine_loop $OUT/c5prof_e/run_kernel_stats.csv | cut -c1-70,150-260
timeout -k 10 300 python3 scripts/c5bench.py > $OUT/c5bench_e.json 2> $OUT/c5bench_e.err; c=$?
echo "c5 exit $c"; cat $OUT/c5bench_e.json
exit $c
