#!/bin/bash
# round 4 session h: round 3's committed quad kernel (51c2b07, 192-B slab rows) at two waves
# per SIMD on grids of two and three workgroups per CU (HW_ID status words), and the current
# kernel at two waves per SIMD, two workgroups per CU, at more shapes and seeds, three runs each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in q192w2c8h q192w2c12h v2h8; do
  for c in "131072 16 7000" "131072 16 1" "40000 16 7000" "131072 10 7000" "40000 3 910" "20001 3 910" "262144 10 5"; do
    set -- $c
    echo "== $lib $c" >> $OUT/hwdiag_h.jsonl
    TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 KB_REPS=3 timeout -k 10 90 python3 scripts/band_hwdiag.py >> $OUT/hwdiag_h.jsonl 2>> $OUT/hwdiag_h.err || exit 1
  done
  echo "$lib done"
done
python3 - <<'PY'
import json
for l in open("gpurun_out/hwdiag_h.jsonl"):
    if l.startswith("=="): print(l.strip()); continue
    d = json.loads(l); print(" rep", d["rep"], "n_bad", d["n_bad"], "max_err", "%.2e" % d["max_err"], "tg_all", d["tg"]["all"][:4], "wave_all", d["wave"]["all"][:4], "cus_used", d["cus_used"], "cus_2tg", d["cus_with_2plus_tg"], "st", d["st"]["all"][:4])
PY
