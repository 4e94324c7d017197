#!/bin/bash
# Standard GPU check: kernel tests, 1-GPU bench, rocprofv3 kernel trace + step timeline.
# Usage: tools/gpu_check.sh [tag] [pytest selection...]
tag=${1:-check}; shift
sel=${@:-tests}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 200 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model transformer --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/step_timeline.py gpurun_out/${tag}_prof/run_results.db --steps 8 > gpurun_out/${tag}_timeline.txt && head -30 gpurun_out/${tag}_timeline.txt
