set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_f32_gpu.py tests/test_gemm_f32_split_gpu.py -k "attention or transformer or vocab" > gpurun_out/t_attn.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_attn.log; exit 1; }
tail -3 gpurun_out/t_attn.log
timeout -k 10 300 python bench.py --model transformer --dtype fp32 --steps 20 --warmup 5 --no-aux --no-f32-compare > gpurun_out/b_fp32.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/b_fp32.log; exit 1; }
grep '^{' gpurun_out/b_fp32.log | tail -1
rm -rf gpurun_out/prof_fp32
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof_fp32 -o run -- python3 bench.py --model transformer --dtype fp32 --steps 8 --warmup 3 --no-aux --no-f32-compare > gpurun_out/prof_fp32.log 2>&1 || { echo PROFFAIL; exit 1; }
DB=$(ls gpurun_out/prof_fp32/*.db gpurun_out/prof_fp32/*/*.db 2>/dev/null | head -1)
python3 tools/step_timeline.py $DB --steps 4 > gpurun_out/prof_fp32_timeline.txt
python3 tools/step_calls.py $DB > gpurun_out/prof_fp32_calls.txt
head -30 gpurun_out/prof_fp32_timeline.txt
rm -rf gpurun_out/prof_fp32
