#!/bin/bash
# Final-loss comparison of the transformer bench across wgrad-group / hip-graph settings.
set -e
mkdir -p gpurun_out
for g in 0 1; do for gr in off on; do
  SPARKMI_WGRAD_GROUP=$g timeout -k 10 120 python bench.py --model transformer --steps 40 --warmup 5 --graph $gr > gpurun_out/lm_${g}_${gr}.json 2> gpurun_out/lm_${g}_${gr}.err
  echo "group=$g graph=$gr $(grep -o '"final_loss": [0-9.]*' gpurun_out/lm_${g}_${gr}.json) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lm_${g}_${gr}.json)"
done; done
