#!/bin/bash
# inlined kernel tails (no scratch), salt sweep with the ReLU-tie hook, small-model benches + profiles
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_seq.sh \
  "200|r4h_small.log|$T tests/test_lstm.py tests/test_cnn.py -m gpu" \
  "400|r4h_salts.log|$T -s tests/test_f32_gpu.py -k across_salts" || exit $?
timeout -k 10 200 python3 bench.py --model cnn > gpurun_out/r4h_bench_cnn.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --model aux > gpurun_out/r4h_bench_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h_prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/r4h_prof_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4h_prof_cnn -o run -- python3 bench.py --model cnn --cnn-steps 100 --warmup 5 > gpurun_out/r4h_prof_cnn.log 2>&1
