set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_f32_gpu.py tests/test_dp_gpu.py > gpurun_out/t_r3b.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error" gpurun_out/t_r3b.log | head; tail -5 gpurun_out/t_r3b.log; exit 1; }
tail -1 gpurun_out/t_r3b.log
bash tools/ab_fp32.sh "SMI_PLANES_ONLY=0 SMI_ATTN_DKDV8=0 SMI_CE_FUSED=0" "SMI_PLANES_ONLY=1 SMI_ATTN_DKDV8=0 SMI_CE_FUSED=0" "SMI_PLANES_ONLY=1 SMI_ATTN_DKDV8=1 SMI_CE_FUSED=0" "SMI_PLANES_ONLY=1 SMI_ATTN_DKDV8=1 SMI_CE_FUSED=1" "SMI_PLANES_ONLY=0 SMI_ATTN_DKDV8=0 SMI_CE_FUSED=0"
