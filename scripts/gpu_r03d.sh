#!/bin/bash
# session d: band timing, config-5 kernel trace + PMC after the cost-form change
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python3 scripts/bandbench.py > $OUT/band_d.json 2> $OUT/band_d.err; c=$?
echo "band exit $c"; cat $OUT/band_d.json; [ $c -eq 0 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5prof_d -o run --output-format csv -- python3 scripts/c5bench.py > $OUT/c5prof_d.json 2> $OUT/c5prof_d.err; c=$?
echo "c5prof exit $c"; cat $OUT/c5prof_d.json; [ $c -eq 0 ] || exit $c
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  C5_K=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/c5pmc_d/p$i -o run -- python3 scripts/c5bench.py > $OUT/c5pmc_d_p$i.json 2> $OUT/c5pmc_d_p$i.err; c=$?
  echo "c5 pmc pass $i exit $c"; [ $c -eq 0 ] || exit $c
done
exit 0
