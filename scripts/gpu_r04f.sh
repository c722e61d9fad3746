#!/bin/bash
# round 4 session f: band-KKT wrong-result diagnosis.  TGMS_BAND_HWID builds (the status word
# of each trajectory = where it ran): v1h the shipped build (one wave per SIMD, no scratch),
# v1sh one wave per SIMD with VGPR spills to scratch memory (AGPR spilling off), v2h8 two
# waves per SIMD (spilling) on a grid of two workgroups per CU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=trajectory_generator_ros2_amd/lib/variants
for lib in v1h v1sh v2h8; do
  for c in "131072 16 7000" "40000 16 7000" "131072 10 7000" "40000 3 910"; do
    set -- $c
    echo "== $lib $c" >> $OUT/hwdiag_f.jsonl
    TGMS_LIB=$V/libtgms_$lib.so KB_B=$1 KB_M=$2 KB_SEED=$3 timeout -k 10 90 python3 scripts/band_hwdiag.py >> $OUT/hwdiag_f.jsonl 2>> $OUT/hwdiag_f.err || exit 1
  done
  echo "$lib done"
done
python3 - <<'PY'
import json
for l in open("gpurun_out/hwdiag_f.jsonl"):
    if l.startswith("=="): print(l.strip()); continue
    d = json.loads(l); print(" rep", d["rep"], "n_bad", d["n_bad"], "max_err", d["max_err"], "slots", d["slots"], "tg_bad", d["tg"]["bad"], "wave_bad", d["wave"]["bad"], "simd_bad", d["simd"]["bad"], "cus_2tg", d["cus_with_2plus_tg"])
PY
