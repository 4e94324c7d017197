#!/bin/bash
# step timelines (fp32 + bf16) with per-call tables, and the bf16 GEMM shape bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/prof_step.sh fp32 gpurun_out/r4e_fp32 || exit $?
python3 tools/step_calls.py gpurun_out/r4e_fp32/run_results.db > gpurun_out/r4e_fp32_calls.txt || exit $?
bash tools/prof_step.sh bf16 gpurun_out/r4e_bf16 || exit $?
python3 tools/step_calls.py gpurun_out/r4e_bf16/run_results.db > gpurun_out/r4e_bf16_calls.txt || exit $?
timeout -k 10 200 python3 tools/bench_gemm_bf16.py > gpurun_out/r4e_gemm_bf16.log 2>&1
