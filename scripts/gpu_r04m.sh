#!/bin/bash
# round 4 session m: config-5 launch shapes with the merged last pass: two classes (default),
# one class at one wave per SIMD (tw1: one launch, no fork/join), boundary 13; then the
# config-5 PMC passes of the default build (profiles/c5_pmc.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for rep in 1 2 3; do
  for lib in default $V/libtgms_tw1.so $V/libtgms_tw13.so; do
    if [ $lib = default ]; then L=""; else L=$lib; fi
    TGMS_LIB=$L timeout -k 10 200 python3 scripts/c5bench.py >> $OUT/c5_m.jsonl 2>> $OUT/c5_m.err || exit 1
  done
done
cut -c1-220 $OUT/c5_m.jsonl
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  C5_K=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/c5pmc_m/p$i -o run -- python3 scripts/c5bench.py > $OUT/c5pmc_m_p$i.json 2> $OUT/c5pmc_m_p$i.err; c=$?
  echo "c5 pmc pass $i exit $c"; [ $c -eq 0 ] || exit $c
done
python3 scripts/c5_pmc.py $OUT/c5pmc_m $OUT/c5_pmc_new.json && cat $OUT/c5_pmc_new.json
