#!/bin/bash
# GPU box: the streaming path's chains swapped (TOWR_GPU_CHAIN_SWAP: FDISC chain on the caller's stream, the
# RangeOfMotion / Dynamic chain on side stream 0 at the default (1) or least (2) priority) against the product
TAG=${1:-r05r}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "two_chains or gait_torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
TOWR_GPU_LAUNCH_LOG=1 TOWR_GPU_CHAIN_SWAP=2 timeout -k 10 100 python tools/gait_ab.py --reps 5 --step-only 2>&1 | grep towr-streams
for i in 1 2 3 4; do
  for SW in 0 1 2; do
    g=$(TOWR_GPU_CHAIN_SWAP=$SW timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only 2>&1 | grep step) || exit 1
    t=$(TOWR_GPU_CHAIN_SWAP=$SW timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque 2>&1 | grep step) || exit 1
    echo "swap $SW gait [$g] torque [$t]" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
