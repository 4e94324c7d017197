#!/bin/bash
# Build the CNN probe (the working tree's) for two versions of the kernel (a git revision vs the
# working tree, each with its own header), stamped and unstamped, into tools/probes/ab_*; run
# tools/cnn_ab_run.sh on the GPU box.
# usage: [BFLAGS=-D...] bash tools/cnn_ab.sh [REV]   (default HEAD)
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
rm -rf /tmp/cnn_ab && mkdir -p /tmp/cnn_ab/a
git archive "$REV" csrc | tar -x -C /tmp/cnn_ab/a
for v in a b; do
  root=$PWD; [ $v = a ] && root=/tmp/cnn_ab/a
  vflags=""; [ $v = b ] && vflags="$BFLAGS"  # BFLAGS: extra -D flags for the working-tree build
  for m in stamp plain; do
    extra=""; [ $m = plain ] && extra="-DCNN_PROBE_NOSTAMP"
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I$root/csrc/include -Wno-unused-value $extra $vflags \
      -DCNN_SRC="\"$root/csrc/kernels/cnn.hip\"" tools/probes/cnn_probe.hip -o tools/probes/ab_${v}_$m &
  done
done
wait
ls tools/probes/ab_*
