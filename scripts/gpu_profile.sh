#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only) for the headline bench
# (a fresh batch every step, 4 sets rotated), folded into profiles/pmc_traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --cpu-seconds 0 --dense-steps 0 --band-steps 0 --sample-traj 0 --config5 0 --config4 0 --cache-resident 0 --host-line 0 --node-line 0 --uniform-large-m 0 --config2 0 $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err; c=$?
  echo "pass $i ($grp) exit $c"
  [ $c -eq 0 ] || exit $c
done
python3 scripts/pmc_traffic.py $OUT B65536_M10_reduced_sets4
