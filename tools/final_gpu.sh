#!/bin/bash
# End-of-round GPU evidence: full GPU suite, 1-GPU bench, fp32 step timeline, stock PyTorch fp32 baseline.
tag=${1:-final}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench.log | cut -c1-600
bash tools/prof_step.sh fp32 gpurun_out/${tag}_prof_fp32 > /dev/null 2>&1 || exit 1
head -24 gpurun_out/${tag}_prof_fp32.txt
timeout -k 10 300 python tools/bench_torch_baseline.py --dtype fp32 > gpurun_out/${tag}_torch_fp32.log 2>&1 || { tail -5 gpurun_out/${tag}_torch_fp32.log; exit 1; }
grep '^{' gpurun_out/${tag}_torch_fp32.log
