#!/bin/bash
cd "$(dirname "$0")"
for shape in "8192 512 512 0" "8192 1536 512 0" "8192 512 512 1" "8192 10000 512 0"; do
  for b in gemm_probe gemm_probe_noepi gemm_probe_nothing; do
    echo -n "$b: "; timeout -k 5 60 ./$b $shape || exit 1
  done
done
