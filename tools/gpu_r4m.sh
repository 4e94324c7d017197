#!/bin/bash
# small-model kernels (MLP LDS weights, LSTM wgrad occupancy, bound inputs): tests, benches,
# profiles; then the default bench (all workloads) and an fp32 step timeline for profiles/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_seq.sh \
  "300|r4m_small.log|$T tests/test_lstm.py tests/test_cnn.py tests/test_mlp_kernel.py tests/test_runner_bind.py tests/test_kernels_gpu.py -m gpu" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4m_prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/r4m_prof_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4m_prof_cnn -o run -- python3 bench.py --model cnn --cnn-steps 100 --warmup 5 > gpurun_out/r4m_prof_cnn.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r4m_bench_all.log 2>&1 || exit $?
bash tools/prof_step.sh fp32 gpurun_out/r4m_fp32 > /dev/null 2>&1 || exit $?
python3 tools/step_calls.py gpurun_out/r4m_fp32/run_results.db --marker adam > gpurun_out/r4m_fp32_calls.txt 2>&1
