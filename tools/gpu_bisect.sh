cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { timeout -k 10 600 python -u -m pytest -q --timeout 250 --timeout-method thread -m gpu "$@" > gpurun_out/bis.log 2>&1; echo "$* :: $(tail -1 gpurun_out/bis.log) :: $(grep -c FAILED gpurun_out/bis.log) $(grep FAILED gpurun_out/bis.log | head -3 | tr '\n' ' ')"; }
run tests/test_f32_gpu.py
run tests/test_cnn.py tests/test_comm_gpu.py tests/test_deferred_gpu.py tests/test_dp_gpu.py tests/test_f32_gpu.py -k "flagship or concat_kv or not f32_gpu"
