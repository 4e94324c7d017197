#!/bin/bash
# write-through hand-offs (CNN / LSTM / MLP / embedding), LSTM LDS-staged MFMA wgrad, the salt sweep
# with ReLU ties taken from the GPU, then the small-model benches and step profiles
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_seq.sh \
  "200|r4g_small.log|$T tests/test_lstm.py tests/test_cnn.py tests/test_mlp_kernel.py -m gpu" \
  "150|r4g_emb.log|$T tests/test_kernels_gpu.py -k 'embedding or optim or adam'" \
  "400|r4g_salts.log|$T -s tests/test_f32_gpu.py -k across_salts" || exit $?
timeout -k 10 200 python3 bench.py --model cnn > gpurun_out/r4g_bench_cnn.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --model aux > gpurun_out/r4g_bench_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/r4g_prof_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_prof_cnn -o run -- python3 bench.py --model cnn --cnn-steps 100 --warmup 5 > gpurun_out/r4g_prof_cnn.log 2>&1 || exit $?
python3 tools/step_calls.py gpurun_out/r4e_fp32/run_results.db --marker adam > gpurun_out/r4e_fp32_calls.txt 2>&1
bash tools/prof_step.sh bf16 gpurun_out/r4e_bf16 || exit $?
python3 tools/step_calls.py gpurun_out/r4e_bf16/run_results.db --marker adam > gpurun_out/r4e_bf16_calls.txt 2>&1
timeout -k 10 200 python3 tools/bench_gemm_bf16.py > gpurun_out/r4e_gemm_bf16.log 2>&1
