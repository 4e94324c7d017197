#!/bin/bash
# Run a sequence of GPU steps; each step has its own timeout; stop at the first step that
# crashed / timed out (exit codes other than 0 and 1).  Usage: tools/gpu_run.sh "cmd1" "cmd2" ...
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for cmd in "$@"; do
  i=$((i+1))
  echo "=== step $i: $cmd" | tee -a gpurun_out/steps.log
  bash -c "$cmd"
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
