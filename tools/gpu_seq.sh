#!/bin/bash
# Run GPU steps in order, each under its own time limit; a test FAILURE (exit 1) moves on to the
# next step, anything else (fault, abort, segfault, timeout) stops the sequence there.
# usage: bash tools/gpu_seq.sh "<secs>|<log>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%|*}; rest=${spec#*|}; log=${rest%%|*}; cmd=${rest#*|}
  echo "[seq] ($secs s) $cmd -> $log"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "[seq] rc=$rc"
  tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[seq] stopping after rc=$rc"; exit $rc; fi
done
