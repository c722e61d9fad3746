#!/bin/bash
# round 4 session n: class boundary 13 (ED 11) as the default: every GPU test, config-5
# timing, config-5 PMC passes; uniform M = 12/14/16: lane kernel vs lane-pair kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_n.log 2>&1; c=$?
echo "pytest exit $c"; tail -2 $OUT/pytest_n.log
[ $c -eq 0 ] || exit $c
for rep in 1 2 3; do
  timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_n.jsonl 2>> $OUT/c5_n.err || exit 1
done
cut -c1-200 $OUT/c5_n.jsonl
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  C5_K=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/c5pmc_n/p$i -o run -- python3 scripts/c5bench.py > $OUT/c5pmc_n_p$i.json 2> $OUT/c5pmc_n_p$i.err; c=$?
  echo "c5 pmc pass $i exit $c"; [ $c -eq 0 ] || exit $c
done
python3 scripts/c5_pmc.py $OUT/c5pmc_n $OUT/c5_pmc_new.json || exit 1
for m in 12 14 16; do
  for lib in default $V/libtgms_lanemax10.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L KB_M=$m KB_ROT=3 KB_K=20 timeout -k 10 300 python3 scripts/kbench.py >> $OUT/lane_n.jsonl 2>> $OUT/lane_n.err || exit 1
  done
done
cut -c1-200 $OUT/lane_n.jsonl
