#!/bin/bash
# round-3 profile session: headline bench, rocprofv3 kernel-trace summaries (headline
# alone and every side line), PMC traffic passes of the headline, config-5 PMC passes,
# and the N = 2 ranks-mode control flow rehearsed over gloo on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
SIDE_OFF="--dense-steps 0 --band-steps 0 --sample-traj 0 --config5 0 --config4 0 --cache-resident 0 --host-line 0 --node-line 0"
timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err; c=$?
echo "bench exit $c"; [ $c -eq 0 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 $SIDE_OFF > $OUT/prof_bench.json 2> $OUT/prof.err; c=$?
echo "rocprof (headline) exit $c"; [ $c -eq 0 ] || exit $c
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_full -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --dense-steps 2 > $OUT/prof_full_bench.json 2> $OUT/prof_full.err; c=$?
echo "rocprof (full) exit $c"; [ $c -eq 0 ] || exit $c
bash scripts/gpu_profile.sh; c=$?
echo "pmc exit $c"; [ $c -eq 0 ] || exit $c
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  C5_K=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/c5pmc_r03/p$i -o run -- python3 scripts/c5bench.py > $OUT/c5pmc_r03_p$i.json 2> $OUT/c5pmc_r03_p$i.err; c=$?
  echo "c5 pmc pass $i exit $c"; [ $c -eq 0 ] || exit $c
done
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 --cpu-seconds 0 --dense-steps 0 --band-steps 0 --host-line 0 --node-line 0 \
    > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err; c=$?
echo "n2 gloo exit $c"
exit $c
