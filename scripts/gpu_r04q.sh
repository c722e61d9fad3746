#!/bin/bash
# round 4 session q: scalar cost accumulator (every launched refinement-loop kernel free of
# scratch): every GPU test, config-5 timing, config-5 PMC passes, smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_q.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_q.log
[ $c -eq 0 ] || exit $c
for rep in 1 2 3; do
  timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_q.jsonl 2>> $OUT/c5_q.err || exit 1
done
cut -c1-200 $OUT/c5_q.jsonl
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  C5_K=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/c5pmc_q/p$i -o run -- python3 scripts/c5bench.py > $OUT/c5pmc_q_p$i.json 2> $OUT/c5pmc_q_p$i.err; c=$?
  echo "c5 pmc pass $i exit $c"; [ $c -eq 0 ] || exit $c
done
python3 scripts/c5_pmc.py $OUT/c5pmc_q $OUT/c5_pmc_new.json || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_q.log 2>&1; c=$?
echo "smoke exit $c"; tail -1 $OUT/smoke_q.log
exit $c
