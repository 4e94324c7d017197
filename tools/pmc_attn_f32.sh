#!/bin/bash
# PMC passes (one counter group per run) over the fp32 attention kernels (tools/ab_attn.py, the
# single-pass backward variant); summaries -> gpurun_out/pmc_attn_f32_*.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcattn_$i -o run -- python3 tools/ab_attn.py --only single_pass > gpurun_out/pmcattn_$i.log 2>&1
  f=$(find gpurun_out/pmcattn_$i -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py "$f" > gpurun_out/pmc_attn_f32_$i.txt
done
