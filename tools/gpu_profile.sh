#!/bin/bash
# Round-end measurement on the GPU box: PMC traffic passes (FETCH_SIZE, WRITE_SIZE, SQ), then the
# full bench (which reads the fresh traffic), then a rocprofv3 kernel-trace --stats run of the same
# bench. Results land in gpurun_out/TAG_*; copy the ones to keep into profiles/.
# Usage: tools/gpu_profile.sh TAG
TAG=${1:-prof}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc.sh ${TAG} 5 "fetch write sq" || exit $?
python3 tools/pmc_traffic.py gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write 4096 gpurun_out/${TAG}_pmc_traffic.json || exit $?
cp gpurun_out/${TAG}_pmc_traffic.json profiles/pmc_traffic.json
python3 tools/pmc_summ.py gpurun_out/${TAG}_sq > gpurun_out/${TAG}_pmc_sq.txt
# the raw per-dispatch counter rows of the engine's kernels (both passes), kept beside the summary
python3 - "$TAG" <<'PY' || exit $?
import csv, glob, sys
tag = sys.argv[1]
with open(f"gpurun_out/{tag}_pmc_raw.csv", "w", newline="") as fo:
    w = None
    for p in ("fetch", "write"):
        for f in glob.glob(f"gpurun_out/{tag}_{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "towr_" not in r["Kernel_Name"]:
                    continue
                row = {k: r.get(k, "") for k in ("Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "Counter_Name", "Counter_Value")}
                if w is None:
                    w = csv.DictWriter(fo, fieldnames=list(row)); w.writeheader()
                w.writerow(row)
PY
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --no-cpu --no-host > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
exit $rc
