#!/bin/bash
# Build the CNN probe for two versions of csrc/kernels/cnn.hip (a git revision vs the working tree),
# stamped and unstamped, into tools/probes/ab_*; run tools/cnn_ab_run.sh on the GPU box.
# usage: bash tools/cnn_ab.sh [REV]   (default HEAD)
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
mkdir -p /tmp/cnn_ab && git show "$REV:csrc/kernels/cnn.hip" > /tmp/cnn_ab/cnn_a.hip
cp csrc/kernels/cnn.hip /tmp/cnn_ab/cnn_b.hip
for v in a b; do
  for m in stamp plain; do
    extra=""; [ $m = plain ] && extra="-DCNN_PROBE_NOSTAMP"
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include -Wno-unused-value $extra \
      -DCNN_SRC="\"/tmp/cnn_ab/cnn_$v.hip\"" tools/probes/cnn_probe.hip -o tools/probes/ab_${v}_$m &
  done
done
wait
ls tools/probes/ab_*
