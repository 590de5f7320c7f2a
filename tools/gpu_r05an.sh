#!/bin/bash
# GPU box: problems per FDISC composer block (RangeOfMotion / Dynamic composer problems per block: product 2, rg4, rg1): parity, then
# gait / gait + Torque steps, one box
TAG=${1:-r05am}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TOWR_GPU_LIB=tools/build/libtowr_gpu_rg4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "gait or stream or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in "" rg4 rg1; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $3}') || exit 1
    echo "${V:-product} gait $g torque $t" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
