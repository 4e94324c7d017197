#!/bin/bash
# Run ONE gpurun call, re-submitting only while the pool reports that nothing ran (exit 3: no box
# free, or an infrastructure "transient" status).  A call that ran and failed is never retried.
# usage: tools/gpu_call.sh <timeout_s> <log> '<command>'
T=$1; LOG=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    echo "[gpu_call] attempt $i: nothing ran (rc=$rc), retrying in 90 s" >> "$LOG.attempts"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
