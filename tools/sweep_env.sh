#!/bin/bash
# Run bench.py (transformer, 1 GPU) once per environment setting given as arguments
# ("VAR=val VAR2=val" strings; "" = defaults) and print ms/step per setting.
# Usage: tools/sweep_env.sh "" "SPARKMI_WGRAD_TARGET=64" ...
mkdir -p gpurun_out
for envs in "$@"; do
  out=$(env $envs timeout -k 10 150 python bench.py --model transformer --steps 30 --warmup 5 2>/dev/null | grep '^{')
  rc=$?
  ms=$(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null)
  echo "[$envs] -> $ms" | tee -a gpurun_out/sweep.log
  if [ $rc -ne 0 ] && [ -z "$ms" ]; then echo "stop: rc=$rc"; exit 1; fi
done
