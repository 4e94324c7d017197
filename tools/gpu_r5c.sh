#!/bin/bash
# CNN in-kernel batch gather (index mode): tests, then the CNN bench (headline step + recipe path)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_loader_gpu.py \
  tests/test_cnn.py tests/test_recipes_gpu.py tests/test_dp_gpu.py tests/test_gemm_bf_gpu.py > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --model cnn --cnn-steps 1875 > gpurun_out/r5c_bench_cnn.log 2>&1 || exit $?
tail -3 gpurun_out/r5c_bench_cnn.log
