#!/bin/bash
# GPU side of tools/cnn_ab.sh: interleaved runs of the two probe builds (bf16 fused step with the weight-gradient helpers)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for v in a b; do
    timeout -k 10 60 tools/probes/ab_${v}_plain 1 1 1 > gpurun_out/cnn_ab_${v}_plain_$r.txt 2>&1 || exit $?
    echo "$v plain run $r: $(grep -E 'graph|kernel' gpurun_out/cnn_ab_${v}_plain_$r.txt | tr '\n' ' ')"
  done
done
for v in a b; do
  timeout -k 10 60 tools/probes/ab_${v}_stamp 1 1 1 > gpurun_out/cnn_ab_${v}_stamp.txt 2>&1 || exit $?
done
paste <(grep phase gpurun_out/cnn_ab_a_stamp.txt) <(grep phase gpurun_out/cnn_ab_b_stamp.txt | awk '{print $5}')
