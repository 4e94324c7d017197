#!/bin/bash
# Two PMC passes over the small-model bench (LSTM/MLP): instruction mix and wait breakdown per kernel
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmclstm_$i -o run -- python3 bench.py --model aux --steps 20 --warmup 5 > gpurun_out/pmclstm_$i.log 2>&1
  f=$(find gpurun_out/pmclstm_$i -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py "$f" > gpurun_out/pmc_lstm_$i.txt
done
