#!/bin/bash
# PMC passes over kbench.py for every variant library (kernel-trace only alongside --pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/kpmc; mkdir -p $OUT
for so in trajectory_generator_ros2_amd/lib/variants/*.so; do
  n=$(basename $so .so); i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    TGMS_LIB=$PWD/$so KB_B=65536 timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$n/p$i -o run -- \
        python3 scripts/kbench.py > $OUT/$n.p$i.json 2> $OUT/$n.p$i.err; c=$?
    echo "$n pass $i exit $c"; [ $c -eq 0 ] || exit $c
  done
done
