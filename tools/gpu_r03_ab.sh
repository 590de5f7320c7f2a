#!/bin/bash
# round 3: gait parity subset, then gait per-kernel timing under environment variants, then a rocprof pass.
# Usage: tools/gpu_r03_ab.sh TAG "VAR=v VAR2=w" "VAR=x" ...
TAG=${1:-r03}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "gait or rotvec or batch_device or gap" > gpurun_out/${TAG}_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "passed|failed|error" gpurun_out/${TAG}_parity.log | tail -3
[ $rc -eq 0 ] || { tail -60 gpurun_out/${TAG}_parity.log; exit $rc; }
timeout -k 10 300 python tools/gait_ab.py --reps 30 > gpurun_out/${TAG}_gait.log 2>&1 || exit $?
for v in "$@"; do
  echo "== $v" >> gpurun_out/${TAG}_gait.log
  env $v timeout -k 10 300 python tools/gait_ab.py --reps 30 >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/single_probe.py gait > gpurun_out/${TAG}_single.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_gait.log; cat gpurun_out/${TAG}_single.log
bash tools/gpu_kprof.sh ${TAG}k || exit $?
