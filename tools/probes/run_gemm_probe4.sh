#!/bin/bash
cd "$(dirname "$0")"
for shape in "8192 512 512 0" "8192 512 512 1" "8192 512 512 2 16"; do
  for b in gemm_probe gemm_probenoepi gemm_probenodma gemm_probenomfma gemm_probenoepi_nodma_nomfma; do
    echo -n "$b: "; timeout -k 5 60 ./$b $shape || exit 1
  done
done
