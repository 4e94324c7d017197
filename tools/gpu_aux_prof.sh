set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_aux
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_aux -o run -- python3 bench.py --model aux --aux-steps 50 --warmup 5 > gpurun_out/prof_aux.log 2>&1 || { echo PROFFAIL; tail -5 gpurun_out/prof_aux.log; exit 1; }
grep '^{' gpurun_out/prof_aux.log | tail -1
find gpurun_out/prof_aux -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/aux_kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/aux_kernel_stats.csv")))
rows.sort(key=lambda r:-float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e3:12.1f} us  {r["Name"][:100]}')
PY
rm -rf gpurun_out/prof_aux
