cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_lstm.py tests/test_kernels_gpu.py tests/test_recipes_gpu.py > gpurun_out/t_r3h.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/t_r3h.log
for v in 1 0 1 0; do
  SMI_ADAM_WIDE=$v timeout -k 10 200 python bench.py --model aux --aux-steps 100 --warmup 10 > gpurun_out/aux_$v.log 2>&1 || exit 1
  echo "ADAM_WIDE=$v $(python -c "import json,sys;d=json.loads([l for l in open('gpurun_out/aux_$v.log') if l.startswith('{')][-1]);print(d['lstm']['ms_per_step'], d['mlp']['ms_per_step'])")"
done
bash tools/ab_fp32.sh "SMI_ADAM_WIDE=0" "SMI_ADAM_WIDE=1" "SMI_ADAM_WIDE=0" "SMI_ADAM_WIDE=1"
