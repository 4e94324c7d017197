#!/bin/bash
# Same-box A/B of fp32 transformer step knobs (box-to-box clocks differ by ~5%: compare only
# within one call).  usage (GPU box): bash tools/ab_fp32.sh "ENV=.. ENV2=.." "ENV=.." ...
set -o pipefail
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 240 python bench.py --model transformer --dtype fp32 --steps 20 --warmup 5 --no-aux \
    --no-f32-compare > gpurun_out/ab_$i.log 2>&1 || { echo "variant $i FAILED: $v"; tail -5 gpurun_out/ab_$i.log; exit 1; }
  echo "$v -> $(grep '^{' gpurun_out/ab_$i.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", d["transformer_fp32"]["final_loss"])')"
done
