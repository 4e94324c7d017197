cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/full_suite.log 2>&1
echo "suite rc=$?"
grep -E "FAILED|ERROR" gpurun_out/full_suite.log | head -20
tail -1 gpurun_out/full_suite.log
timeout -k 10 120 python tools/bench_lstm.py || exit 1
bash tools/gpu_aux_prof.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit 1
tail -1 gpurun_out/bench_full.log | cut -c1-1500
