#!/bin/bash
cd "$(dirname "$0")"
for shape in "8192 512 512 0" "8192 1024 512 0" "8192 512 1024 0" "8192 1536 512 0" "8192 512 512 1" "8192 512 1024 1" "8192 1024 512 1" "8192 10000 512 0"; do
  for bm in 64 128; do
    for ns in 2 4; do
      echo -n "BM=$bm NS=$ns "; SMI_GEMM_BM=$bm SMI_GEMM_NS=$ns timeout -k 5 60 ./gemm_probe $shape || exit 1
    done
  done
done
