set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_lstm.py tests/test_f32_gpu.py -k "lstm or overlap or transformer" > gpurun_out/t_r3c.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|assert" gpurun_out/t_r3c.log | head; tail -5 gpurun_out/t_r3c.log; exit 1; }
tail -1 gpurun_out/t_r3c.log
timeout -k 10 120 python tools/bench_lstm.py
bash tools/gpu_aux_prof.sh
