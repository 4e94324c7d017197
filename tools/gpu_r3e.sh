cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_lstm.py > gpurun_out/t_lstm.log 2>&1; tail -1 gpurun_out/t_lstm.log
timeout -k 10 120 python tools/bench_lstm.py
timeout -k 10 300 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_f32_gpu.py -k "flagship" > gpurun_out/t_flag.log 2>&1; tail -1 gpurun_out/t_flag.log; grep "^E  .*Assertion" gpurun_out/t_flag.log | cut -c1-900
