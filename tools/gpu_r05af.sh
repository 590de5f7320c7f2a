#!/bin/bash
# GPU box: 1 KB-aligned store trips (TOWR_ALIGN_TRIPS variant): the write probe, the parity tests with the variant, then
# the headline / gait / gait + Torque steps against the product, one box
TAG=${1:-r05af}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/build/stride_probe > gpurun_out/${TAG}_probe.log 2>&1 || exit 1
cat gpurun_out/${TAG}_probe.log
TOWR_GPU_LIB=tools/build/libtowr_gpu_align.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in "" align; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    h=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 $L 2>&1 | grep -E "^\\S+ +(range_of_motion\\+|dynamic|small|step)" | awk '{print $2, $3}' | tr '\n' ' ') || exit 1
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $3}') || exit 1
    echo "${V:-product} headline [$h] gait $g torque $t" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
