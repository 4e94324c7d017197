#!/bin/bash
# fp32 split-bf16 GEMM check on the GPU box: precision test, per-shape time/error, fp32 step bench.
mkdir -p gpurun_out
tag=${1:-split}
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f32_split_gpu.py > gpurun_out/${tag}_test.log 2>&1 || { tail -30 gpurun_out/${tag}_test.log; exit 1; }
tail -1 gpurun_out/${tag}_test.log
timeout -k 10 200 python tools/f32_split_check.py > gpurun_out/${tag}_check.log 2>&1 || { tail -20 gpurun_out/${tag}_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_check.log
for a in ${ALGOS:-6}; do
SMI_F32_ALGO=$a timeout -k 10 200 python bench.py --model transformer --dtype fp32 --no-aux > gpurun_out/${tag}_bench$a.log 2>&1 || { tail -20 gpurun_out/${tag}_bench$a.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench$a.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('algo $a step', d['ms_per_step'], 'ms', d['value'], 'samples/s', 'loss', d['transformer_fp32']['final_loss'])"
done
