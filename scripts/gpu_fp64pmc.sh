#!/bin/bash
# FP64 instruction counters (rocprofv3 --pmc, one group per pass, --kernel-trace only)
# and HBM bytes for the three solve methods at config 3 (scripts/kbench.py), folded
# into gpurun_out/fp64pmc/summary.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/fp64pmc
mkdir -p $OUT
for meth in 0 1 2; do
  B=65536; K=5
  [ $meth = 1 ] && B=8192 && K=2
  i=0
  for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    KB_METHOD=$meth KB_B=$B KB_K=$K timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d $OUT/m${meth}_p$i -o run -- python3 scripts/kbench.py > $OUT/m${meth}_p$i.json 2> $OUT/m${meth}_p$i.err; c=$?
    echo "method $meth pass $i ($grp) exit $c"
    [ $c -eq 0 ] || exit $c
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
lines = []
for meth, kname, B in ((0, "k_lane_uniform", 65536), (1, "k_dense_gj", 8192), (2, "k_band_kkt", 65536)):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/m{meth}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in acc.items()}
    lines.append(f"{kname} (B = {B}, M = 10), mean per dispatch")
    for k in sorted(mean):
        lines.append(f"  {k:26s} {mean[k]:18.1f}")
    f64 = sum(mean.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
    flops = 64 * (mean.get("SQ_INSTS_VALU_ADD_F64", 0) + mean.get("SQ_INSTS_VALU_MUL_F64", 0) + 2 * mean.get("SQ_INSTS_VALU_FMA_F64", 0))
    hbm = mean.get("FETCH_SIZE", 0) * 1024 * 2 + mean.get("WRITE_SIZE", 0) * 1024
    lines.append(f"  FP64 wave-instructions {f64:.0f}; executed FP64 flop (64 lanes, FMA = 2) {flops:.3e} = {flops / B:.0f} per trajectory")
    lines.append(f"  HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) {hbm:.3e} = {hbm / B:.0f} per trajectory")
open(f"{out}/summary.txt", "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
PY
