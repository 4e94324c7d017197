#!/bin/bash
# kernel trace of the LSTM / MLP benches -> the last step of each (tools/kernel_tail.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_aux
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/prof_aux -o run -- \
  python3 bench.py --model aux --aux-steps 64 --warmup 5 > gpurun_out/prof_aux.log 2>&1 || exit $?
{ echo "== LSTM step (last launches up to the last lstm_bwd + tail)"
  python3 tools/kernel_tail.py gpurun_out/prof_aux/run_results.db 'lstm_bwd' 12 8
  echo "== MLP (last launches)"
  python3 tools/kernel_tail.py gpurun_out/prof_aux/run_results.db 'mlp_' 12 0
} > gpurun_out/prof_aux.txt 2>&1
rm -f gpurun_out/prof_aux/run_results.db
cat gpurun_out/prof_aux.txt
