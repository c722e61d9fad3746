#!/bin/bash
# Config-5 per-call overhead A/Bs (round 6): scripts/c5bench.py under each setting,
# alternating, REPS rounds; one JSON line per run prefixed with the setting.
#   bash scripts/c5_stream_ab.sh OUT REPS SETTING [SETTING ...]   (SETTING: base or K=V,K=V)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; REPS=$2; shift 2
: > "$OUT"
for r in $(seq "$REPS"); do
  for v in "$@"; do
    envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
    line=$(env $envs timeout -k 10 120 python3 scripts/c5bench.py) || { echo "run $v failed"; exit 1; }
    echo "{\"variant\": \"$v\", \"run\": $r, \"result\": $line}" >> "$OUT"
  done
done
cat "$OUT"
