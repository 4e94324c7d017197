#!/bin/bash
# LSTM: fused-CE step computes the head at the last step only; tests, aux bench, aux timeline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_lstm.py \
  tests/test_recipes_gpu.py > gpurun_out/r5h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5h_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --model aux > gpurun_out/r5h_bench_aux.log 2>&1 || exit $?
tail -1 gpurun_out/r5h_bench_aux.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (v.get('ms_per_step'), v.get('samples_per_s')) for k, v in d.get('extra', d).items() if isinstance(v, dict)})"
bash tools/prof_aux.sh > /dev/null 2>&1 || exit $?
head -8 gpurun_out/prof_aux.txt
