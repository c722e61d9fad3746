#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/icache; mkdir -p $OUT
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/bandbench.py > $OUT/p$i.json 2> $OUT/p$i.err; c=$?
  echo "pass $i exit $c"; tail -3 $OUT/p$i.err; [ $c -eq 0 ] || exit $c
done
