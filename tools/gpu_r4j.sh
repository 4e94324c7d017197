#!/bin/bash
# fp32 step A/B of the attention backward epilogue / stagger inside the real step (cross-attention
# dK/dV go to the 6-layer concatenated kv gradient, row stride 6144)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "base|" "aebwd|SMI_ATTN_AE_BWD=1" "stag|SMI_ATTN_STAGGER=1" "aebwd_stag|SMI_ATTN_AE_BWD=1 SMI_ATTN_STAGGER=1"; do
  name=${v%%|*}; envs=${v#*|}
  env $envs timeout -k 10 200 python3 bench.py --model transformer --dtype fp32 --steps 20 --warmup 5 --no-aux --no-f32-compare > gpurun_out/r4j_bench_$name.log 2>&1 || exit $?
  grep '^{' gpurun_out/r4j_bench_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
done
SMI_ATTN_AE_BWD=1 bash tools/prof_step.sh fp32 gpurun_out/r4j_fp32_aebwd > /dev/null 2>&1 || exit $?
python3 tools/step_calls.py gpurun_out/r4j_fp32_aebwd/run_results.db --marker adam > gpurun_out/r4j_fp32_aebwd_calls.txt 2>&1
