#!/bin/bash
# attention variant diagnostics + per-kernel profiles of the A/B variants
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_seq.sh \
  "120|r4b_dbg.log|python tools/dbg_attn_ab.py" \
  "120|r4b_ab.log|python tools/ab_attn.py" \
  "300|r4b_salts.log|python -u -m pytest -v --timeout 280 --timeout-method thread tests/test_f32_gpu.py -k across_salts"
for v in base ae ae+stagger ae+stagger+fwd8s; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b_prof_$v -o run -- python3 tools/ab_attn.py --only "$v" > gpurun_out/r4b_prof_$v.log 2>&1 || exit $?
done
