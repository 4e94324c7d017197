cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/full_suite.log 2>&1
echo "suite rc=$?"
grep -E "FAILED|ERROR" gpurun_out/full_suite.log | head -20
tail -2 gpurun_out/full_suite.log
