#!/bin/bash
# Kernel timeline of the transformer step (rocprofv3 kernel trace -> tools/step_timeline.py).
# usage (on the GPU box): bash tools/prof_step.sh bf16|fp32 [outdir]
set -e
DT=${1:-bf16}
OUT=${2:-gpurun_out/prof_$DT}
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
rm -rf "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT" -o run -- \
  python3 bench.py --model transformer --dtype "$DT" --steps 10 --warmup 3 --no-aux --no-f32-compare > "$OUT.log" 2>&1
python3 tools/step_timeline.py "$OUT/run_results.db" --steps 4 --marker multi_copy_kernel > "$OUT.txt"
grep '^{' "$OUT.log" | tail -1
head -40 "$OUT.txt"
