#!/bin/bash
# MLP multi-step kernel (+ index mode): tests, then the aux bench (LSTM / MLP)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_mlp_kernel.py \
  tests/test_loader_gpu.py tests/test_recipes_gpu.py > gpurun_out/r5f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --model aux --aux-steps 2000 > gpurun_out/r5f_bench_aux.log 2>&1 || exit $?
tail -1 gpurun_out/r5f_bench_aux.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (v.get('ms_per_step'), v.get('samples_per_s')) for k, v in d.get('extra', d).items() if isinstance(v, dict)})"
bash tools/prof_aux.sh > /dev/null 2>&1 || exit $?
head -50 gpurun_out/prof_aux.txt
