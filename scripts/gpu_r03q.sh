#!/bin/bash
# end-of-round-3 session: smoke, the whole -m gpu suite, the headline bench, rocprofv3
# kernel-trace summaries (headline alone, every side line), PMC traffic of the headline,
# PMC of the band-KKT kernel (bandbench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_q.log 2>&1; c=$?
echo "smoke exit $c"; tail -1 $OUT/smoke_q.log; [ $c -eq 0 ] || exit $c
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest_q.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_q.log
[ $c -eq 0 ] || exit $c
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 > $OUT/bench_q.json 2> $OUT/bench_q.err; c=$?
echo "bench exit $c"; [ $c -eq 0 ] || exit $c
SIDE_OFF="--dense-steps 0 --band-steps 0 --sample-traj 0 --config5 0 --config4 0 --cache-resident 0 --host-line 0 --node-line 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_q -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 $SIDE_OFF > $OUT/prof_q_bench.json 2> $OUT/prof_q.err; c=$?
echo "rocprof (headline) exit $c"; [ $c -eq 0 ] || exit $c
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_q_full -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --dense-steps 2 > $OUT/prof_q_full_bench.json 2> $OUT/prof_q_full.err; c=$?
echo "rocprof (full) exit $c"; [ $c -eq 0 ] || exit $c
bash scripts/gpu_profile.sh; c=$?
echo "pmc exit $c"; [ $c -eq 0 ] || exit $c
bash scripts/gpu_bandpmc.sh; c=$?
echo "band pmc exit $c"
exit $c
