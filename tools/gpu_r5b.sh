#!/bin/bash
# bf16 256x128 GEMM: tests, in-step A/B against the 128x128 kernel, bf16 step timeline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_bf_gpu.py \
  tests/test_gemm_gpu.py tests/test_mlp_kernel.py > gpurun_out/r5b_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/ab_step.py "C:gemm_bf256=1,0" --dtype bf16 --rounds 2 > gpurun_out/r5b_ab_bf256.log 2>&1 || exit $?
tail -2 gpurun_out/r5b_ab_bf256.log
bash tools/prof_step.sh bf16 gpurun_out/r5b_bf16 > /dev/null 2>&1 || exit $?
python3 tools/step_calls.py gpurun_out/r5b_bf16/run_results.db --marker adam > gpurun_out/r5b_bf16_calls.txt 2>&1
rm -f gpurun_out/r5b_bf16/run_results.db
head -30 gpurun_out/r5b_bf16.txt
