#!/bin/bash
# round 3: streaming RangeOfMotion / Dynamic — gait parity subset, then per-kernel timing (tile path A/B)
TAG=${1:-r03b}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "gait or rotvec or batch_device" > gpurun_out/${TAG}_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "passed|failed|error" gpurun_out/${TAG}_parity.log | tail -3
[ $rc -eq 0 ] || { tail -60 gpurun_out/${TAG}_parity.log; exit $rc; }
timeout -k 10 300 python tools/gait_ab.py --reps 30 > gpurun_out/${TAG}_gait.log 2>&1 || exit $?
TOWR_GPU_GAIT_TILES=1 timeout -k 10 300 python tools/gait_ab.py --reps 30 >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
timeout -k 10 300 python tools/gait_ab.py --reps 30 --rotvec >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
timeout -k 10 300 python tools/single_probe.py gait > gpurun_out/${TAG}_single.log 2>&1 || exit $?
cat gpurun_out/${TAG}_gait.log gpurun_out/${TAG}_single.log
