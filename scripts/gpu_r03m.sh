#!/bin/bash
# session m: quad band-KKT ablations (forward only, forward without slab stores) + PMC
# traffic / instruction counters of the full kernel (scripts/bandbench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT/bandpmc
V=trajectory_generator_ros2_amd/lib/variants
for lib in default $V/libtgms_noback.so $V/libtgms_nobacknostore.so; do
  if [ $lib = default ]; then L=""; else L=$lib; fi
  TGMS_LIB=$L timeout -k 10 120 python3 scripts/bandbench.py >> $OUT/band_m.jsonl 2>> $OUT/band_m.err || exit 1
done
cat $OUT/band_m.jsonl
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/bandpmc/p$i -o run -- \
      python3 scripts/bandbench.py > $OUT/bandpmc/p$i.json 2> $OUT/bandpmc/p$i.err; c=$?
  echo "pass $i ($grp) exit $c"
  [ $c -eq 0 ] || exit $c
done
