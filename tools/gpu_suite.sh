#!/bin/bash
# full GPU suite (one process), then a 1-GPU bench; logs under gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/suite.log | head -20; tail -2 gpurun_out/suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > gpurun_out/suite_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/suite_bench.log | cut -c1-300
