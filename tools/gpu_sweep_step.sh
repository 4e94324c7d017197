#!/bin/bash
# in-step A/B of kernel-selection switches on the fp32 transformer step (one box, one call):
# isolated kernel benches mispredicted the step before (attention backward epilogue)
# usage: bash tools/gpu_sweep_step.sh "name|ENV=1 ENV2=0" ...   (base first and last)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%|*}; envs=${v#*|}
  env $envs timeout -k 10 200 python3 bench.py --model transformer --dtype fp32 --steps 12 --warmup 4 --no-aux --no-f32-compare > gpurun_out/sweep_$name.log 2>&1 || exit $?
  grep '^{' gpurun_out/sweep_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], flush=True)"
done
