#!/bin/bash
# CNN conv_mfma register tables + wgrad two-step pipelining: tests, phase probe, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_cnn.py \
  tests/test_loader_gpu.py > gpurun_out/r5e_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5e_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/probes/cnn_probe 1 1 > gpurun_out/r5e_probe_bf16_fused.txt 2>&1 || exit $?
tail -25 gpurun_out/r5e_probe_bf16_fused.txt
timeout -k 10 300 python3 bench.py --model cnn --cnn-steps 1875 > gpurun_out/r5e_bench_cnn.log 2>&1 || exit $?
tail -1 gpurun_out/r5e_bench_cnn.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k]['ms_per_step'] for k in ('cnn','cnn_fp32','cnn_recipe_path')})"
