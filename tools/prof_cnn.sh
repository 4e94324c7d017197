#!/bin/bash
# kernel trace of the CNN benches (bound-graph step, fp32, recipe path) -> per-kernel table
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_cnn
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof_cnn -o run -- \
  python3 bench.py --model cnn --cnn-steps 64 --warmup 5 > gpurun_out/prof_cnn.log 2>&1 || exit $?
python3 tools/cnn_timeline.py gpurun_out/prof_cnn/run_results.db > gpurun_out/prof_cnn.txt 2>&1
rm -f gpurun_out/prof_cnn/run_results.db
cat gpurun_out/prof_cnn.txt | head -60
