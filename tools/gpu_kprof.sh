#!/bin/bash
# per-kernel rocprofv3 stats of the gait workload (tools/gait_ab.py): TAG [extra gait_ab args]
TAG=${1:-kp}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 tools/gait_ab.py --reps 30 "$@" > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
python3 - gpurun_out/${TAG}_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "towr" not in n: continue
    print(f"{float(r['AverageNs'])/1e3:9.1f} us avg  {int(r['Calls']):6d} calls  {n[:110]}")
PY
exit $rc
