#!/bin/bash
# CNN tail: A/B against HEAD (probe, helpers on), the CNN GPU tests, then the CNN bench
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/cnn_ab_run.sh > gpurun_out/r5m_ab.txt 2>&1 || { cat gpurun_out/r5m_ab.txt; exit 1; }
cat gpurun_out/r5m_ab.txt | head -4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_cnn.py tests/test_loader_gpu.py tests/test_dp_gpu.py > gpurun_out/r5m_tests.log 2>&1 || { tail -30 gpurun_out/r5m_tests.log; exit 1; }
tail -1 gpurun_out/r5m_tests.log
timeout -k 10 300 python bench.py --model cnn --dtype both --steps 20 --warmup 5 --no-aux > gpurun_out/r5m_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r5m_bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ('cnn','cnn_fp32','cnn_recipe_path'): print(k, d[k]['ms_per_step'])"; exit $rc
