#!/bin/bash
# full GPU suite, then small-model profiles, the default bench (all workloads) and an fp32 step
# timeline for profiles/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/val_suite.log 2>&1
rc=$?; tail -3 gpurun_out/val_suite.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/val_prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/val_prof_aux.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/val_prof_cnn -o run -- python3 bench.py --model cnn --cnn-steps 100 --warmup 5 > gpurun_out/val_prof_cnn.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/val_bench_all.log 2>&1 || exit $?
grep '^{' gpurun_out/val_bench_all.log | cut -c1-300
bash tools/prof_step.sh fp32 gpurun_out/val_fp32 > /dev/null 2>&1 || exit $?
python3 tools/step_calls.py gpurun_out/val_fp32/run_results.db --marker adam > gpurun_out/val_fp32_calls.txt 2>&1
