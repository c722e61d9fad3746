#!/bin/bash
# round-3 session b: probe v2, the remaining new tests, config-4 full-size trace, config-5 trace + PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./scripts/micro/occstore > $OUT/occstore2.txt 2>&1; c=$?
echo "occstore exit $c"; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_edges.py tests/test_gpu_full_configs.py > $OUT/pytest_b.log 2>&1; c=$?
echo "pytest exit $c"; tail -3 $OUT/pytest_b.log
[ $c -eq 0 ] || [ $c -eq 1 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4prof -o run --output-format csv -- python3 scripts/c4full.py > $OUT/c4full.json 2> $OUT/c4full.err; c=$?
echo "c4 exit $c"; cat $OUT/c4full.json; [ $c -eq 0 ] || exit $c
timeout -k 10 300 python3 scripts/c5bench.py > $OUT/c5bench.json 2> $OUT/c5bench.err; c=$?
echo "c5 exit $c"; cat $OUT/c5bench.json; [ $c -eq 0 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5prof -o run --output-format csv -- python3 scripts/c5bench.py > $OUT/c5prof.json 2> $OUT/c5prof.err; c=$?
echo "c5prof exit $c"; [ $c -eq 0 ] || exit $c
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  C5_K=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/c5pmc/p$i -o run -- python3 scripts/c5bench.py > $OUT/c5pmc_p$i.json 2> $OUT/c5pmc_p$i.err; c=$?
  echo "c5 pmc pass $i exit $c"; [ $c -eq 0 ] || exit $c
done
exit 0
