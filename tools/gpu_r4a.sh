#!/bin/bash
# round-4 validation batch (one GPU call): new kernels' tests first, then the bench, then the
# multi-process tests
T="python -u -m pytest -v --timeout 240 --timeout-method thread"
bash tools/gpu_seq.sh \
  "200|r4_lstm.log|$T tests/test_lstm.py -m gpu" \
  "200|r4_cnn.log|$T tests/test_cnn.py -m gpu" \
  "150|r4_emb.log|$T tests/test_kernels_gpu.py -k embedding" \
  "400|r4_f32.log|$T tests/test_f32_gpu.py -k 'attention or step_matches or concat_kv or across_salts'" \
  "120|r4_abattn.log|python tools/ab_attn.py" \
  "200|r4_bench.log|python bench.py --steps 20 --warmup 5" \
  "300|r4_comm.log|$T tests/test_comm_gpu.py" \
  "420|r4_dp.log|python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_dp_gpu.py" \
  "300|r4_benchtest.log|$T tests/test_bench.py -m gpu"
