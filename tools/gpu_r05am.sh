#!/bin/bash
# GPU box: the RangeOfMotion / Dynamic / TQDISC composers' value phase unrolled (TOWR_GS_VAL_UNROLL: product 4, vu2, vu1 =
# round 4's loop): parity of the streaming path, then gait / gait + Torque steps, one box
TAG=${1:-r05am}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "gait or stream or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in "" vu1 vu2; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $3}') || exit 1
    echo "${V:-product} gait $g torque $t" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
