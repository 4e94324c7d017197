#!/bin/bash
# ablation of the production GEMM on the transformer shapes: full / no-epilogue / no-DMA /
# no-MFMA / nothing, at BM 64 and 128 (SMI_GEMM_BM) — where does an 8192 x 512 x 512 GEMM spend its time
cd "$(dirname "$0")"
for shape in "8192 512 512 0" "8192 1536 512 0" "8192 512 1024 0" "8192 512 512 1" "8192 512 512 2 16"; do
  for bm in 64 128; do
    for b in gemm_probe gemm_probenoepi gemm_probenodma gemm_probenomfma gemm_probenoepi_nodma_nomfma; do
      echo -n "BM=$bm $b: "; SMI_GEMM_BM=$bm timeout -k 5 60 ./$b $shape || exit 1
    done
  done
done
