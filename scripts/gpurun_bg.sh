#!/bin/bash
# gpurun_bg.sh LOG TIMEOUT CMD: one gpurun call; re-queued only while no box/slot is
# free (exit 3, nothing ran, nothing charged) or the box was lost before the command
# started (status "transient"); never re-runs a command that ran.
log=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1; rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then sleep 150; continue; fi
  break
done
echo "[gpurun_bg] rc=$rc attempts=$i" >> "$log"
