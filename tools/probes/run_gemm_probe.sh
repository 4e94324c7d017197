#!/bin/bash
# ablation table for tools/probes/gemm_probe*: full / no-DMA / no-MFMA / neither, NS=2 and NS=4
cd "$(dirname "$0")"
for shape in "8192 512 512 0" "8192 1536 512 0" "8192 512 1024 0" "8192 512 512 1" "8192 512 512 2 8" "8192 10000 512 0"; do
  for ns in 2 4; do
    for b in gemm_probe gemm_probedgemm_probe_nodma gemm_probedgemm_probe_nomfma gemm_probedgemm_probe_nodmadgemm_probe_nomfma; do
      echo -n "NS=$ns $b: "; SMI_GEMM_NS=$ns timeout -k 5 60 ./$b $shape || exit 1
    done
  done
done
