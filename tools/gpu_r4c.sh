#!/bin/bash
# small-model regressions: tests, then per-kernel stats of the CNN and LSTM / MLP steps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -v --timeout 240 --timeout-method thread"
bash tools/gpu_seq.sh \
  "200|r4c_small.log|$T tests/test_lstm.py tests/test_cnn.py -m gpu" \
  "150|r4c_emb.log|$T tests/test_kernels_gpu.py -k embedding" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c_prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/r4c_prof_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c_prof_cnn -o run -- python3 bench.py --model cnn --cnn-steps 100 --warmup 5 > gpurun_out/r4c_prof_cnn.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --model cnn > gpurun_out/r4c_bench_cnn.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --model aux > gpurun_out/r4c_bench_aux.log 2>&1
