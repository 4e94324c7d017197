#!/bin/bash
# embedding plan beside the LSTM forward, parallel partial loads (LSTM wgrad, CNN tail): benches,
# profiles, then the whole GPU suite
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash tools/gpu_seq.sh "200|r4i_small.log|$T tests/test_lstm.py tests/test_cnn.py -m gpu" || exit $?
timeout -k 10 200 python3 bench.py --model cnn > gpurun_out/r4i_bench_cnn.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --model aux > gpurun_out/r4i_bench_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i_prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/r4i_prof_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i_prof_cnn -o run -- python3 bench.py --model cnn --cnn-steps 100 --warmup 5 > gpurun_out/r4i_prof_cnn.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4i_suite.log 2>&1
