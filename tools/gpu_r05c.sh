#!/bin/bash
# GPU box: gait parity, then same-box A/B of the gait step: records-first schedule (default) vs the round-4 chains
# (TOWR_GPU_GAIT_SCHED=chain), plain and + Torque; phase stamps of the new schedule
TAG=${1:-r05c}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for S in rec chain; do
    for T in "" --torque; do
      echo "sched=$S $T" >> gpurun_out/${TAG}_ab.log
      TOWR_GPU_GAIT_SCHED=$S timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_stamps_step.log 2>&1 || exit $?
timeout -k 10 200 python tools/stamps.py --torque > gpurun_out/${TAG}_stamps_torque.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_stamps_*.log
