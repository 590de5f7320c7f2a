#!/bin/bash
# GPU box: gait parity, then same-box A/B of the gait step schedules (TOWR_GPU_GAIT_SCHED): chain (round 4),
# rec (records first, one chunk), pipe2 / pipe4 / pipe8, plain and + Torque
TAG=${1:-r05d}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for S in chain rec pipe2 pipe4 pipe8; do
    for T in "" --torque; do
      echo "sched=$S $T $(TOWR_GPU_GAIT_SCHED=$S timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
    done
  done
done
cat gpurun_out/${TAG}_ab.log
