#!/bin/bash
# session f: joint-axes solve for the one-wave kernels: parity + timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_full_configs.py > $OUT/pytest_f.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_f.log
[ $c -eq 0 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5prof_f -o run --output-format csv -- python3 scripts/c5bench.py > $OUT/c5prof_f.json 2> $OUT/c5prof_f.err; c=$?
echo "c5prof exit $c"; cat $OUT/c5prof_f.json; grep refine_loop $OUT/c5prof_f/run_kernel_stats.csv | cut -c1-70,150-260
timeout -k 10 300 python3 scripts/c5bench.py > $OUT/c5bench_f.json 2> $OUT/c5bench_f.err; c=$?
echo "c5 exit $c"; cat $OUT/c5bench_f.json
exit $c
