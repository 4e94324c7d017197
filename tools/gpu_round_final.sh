#!/bin/bash
# End-of-round GPU pass on the final tree: smoke(), the full GPU suite, the default bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/final_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/final_suite.log | head -20; tail -1 gpurun_out/final_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > gpurun_out/final_bench.log 2>&1 || exit $?
tail -1 gpurun_out/final_bench.log | cut -c1-200
