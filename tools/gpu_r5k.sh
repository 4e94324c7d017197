#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_cnn.py \
  tests/test_loader_gpu.py tests/test_dp_gpu.py > gpurun_out/r5k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/probes/cnn_probe 1 1 1 > gpurun_out/r5k_probe_bf16_helpers.txt 2>&1 || exit $?
grep -v "^img" gpurun_out/r5k_probe_bf16_helpers.txt | grep -v "tables"
for dt in bf16 fp32; do
  timeout -k 10 300 python3 tools/ab_cnn.py "sparkmi.ops.cnn:WGRAD_HELPERS=1,0" --dtype $dt > gpurun_out/r5k_ab_$dt.log 2>&1 || exit $?
  tail -2 gpurun_out/r5k_ab_$dt.log
done
