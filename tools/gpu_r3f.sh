cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 250 --timeout-method thread tests/test_f32_gpu.py tests/test_gemm_sp_gpu.py tests/test_lstm.py > gpurun_out/t_r3f.log 2>&1
echo "tests rc=$?"; grep -E "FAILED" gpurun_out/t_r3f.log | head; tail -1 gpurun_out/t_r3f.log
timeout -k 10 60 ./tools/probes/lstm_fwd_probe
bash tools/ab_fp32.sh "SMI_FFN_MASK=0" "SMI_FFN_MASK=1" "SMI_FFN_MASK=0" "SMI_FFN_MASK=1" "SMI_FFN_MASK=0" "SMI_FFN_MASK=1"
