#!/bin/bash
# fp32 and bf16 transformer step timelines (per family, per call, absolute call times) for profiles/
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/prof_step.sh fp32 gpurun_out/r5_fp32 > gpurun_out/r5_fp32_head.txt 2>&1 || { tail -20 gpurun_out/r5_fp32.log; exit 1; }
python3 tools/step_calls.py gpurun_out/r5_fp32/run_results.db --marker adam > gpurun_out/r5_fp32_calls.txt 2>&1 && python3 tools/step_calls.py gpurun_out/r5_fp32/run_results.db --marker adam --abs > gpurun_out/r5_fp32_abs.txt 2>&1
bash tools/prof_step.sh bf16 gpurun_out/r5_bf16 > gpurun_out/r5_bf16_head.txt 2>&1 || { tail -20 gpurun_out/r5_bf16.log; exit 1; }
python3 tools/step_calls.py gpurun_out/r5_bf16/run_results.db --marker adam > gpurun_out/r5_bf16_calls.txt 2>&1 && python3 tools/step_calls.py gpurun_out/r5_bf16/run_results.db --marker adam --abs > gpurun_out/r5_bf16_abs.txt 2>&1
rm -rf gpurun_out/r5_fp32 gpurun_out/r5_bf16
head -3 gpurun_out/r5_fp32.txt gpurun_out/r5_bf16.txt
