cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r5_base_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r5_base_bench.log | cut -c1-400
bash tools/prof_step.sh fp32 gpurun_out/r5_base_fp32 > /dev/null 2>&1 || exit $?
python3 tools/step_calls.py gpurun_out/r5_base_fp32/run_results.db --marker adam > gpurun_out/r5_base_fp32_calls.txt 2>&1
rm -rf gpurun_out/r5_base_fp32/run_results.db
