#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ldspmc; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
for so in trajectory_generator_ros2_amd/lib/variants/libtgms_nc_nostore.so trajectory_generator_ros2_amd/lib/variants/libtgms_w1.so; do
  n=$(basename $so .so); i=0
  for grp in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" "SQ_INSTS_LDS SQ_LDS_MEM_VIOLATIONS SQ_WAIT_INST_LDS SQ_INSTS_SMEM" "SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    TGMS_LIB=$PWD/$so timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/$n/p$i -o run -- \
        python3 scripts/kbench.py > $OUT/$n.p$i.json 2> $OUT/$n.p$i.err; c=$?
    echo "$n pass $i exit $c"
  done
done
exit 0
