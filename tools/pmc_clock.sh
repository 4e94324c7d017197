#!/bin/bash
# One PMC pass over a command: clock cycles (GRBM_COUNT / GRBM_GUI_ACTIVE), MFMA instruction count
# and MFMA-busy cycles per kernel, with kernel durations (kernel trace) -> effective clock and
# matrix-pipe utilisation.  Usage: tools/pmc_clock.sh <outdir> <python script + args>
set -e
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d "$out" -o run -- python3 "$@" > "$out.log" 2>&1
