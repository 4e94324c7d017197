#!/bin/bash
# round-5 check: the pruned attention / plane-GEMM kernels, the DP CNN fast step, the fixed loader
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_loader_gpu.py tests/test_dp_gpu.py::test_cnn_dp_fused_step_matches_single_process \
  tests/test_bench.py::test_bench_cnn_two_ranks_on_the_gpu tests/test_f32_gpu.py tests/test_gemm_sp_gpu.py \
  > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5a_tests.log; grep "cnn bf16 ms/step" gpurun_out/r5a_tests.log; exit $rc
