# round-end validation on one GPU: LSTM probe, full GPU suite, smoke, 1-GPU bench, aux kernel profile
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/probes/lstm_fwd_probe || exit 1
bash tools/gpu_full.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final.log 2>&1; echo "bench rc=$?"; grep '^{' gpurun_out/bench_final.log | tail -1 | cut -c1-400
bash tools/gpu_aux_prof.sh
