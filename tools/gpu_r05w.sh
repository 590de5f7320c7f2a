#!/bin/bash
# GPU box: the -m gpu suite, then the headline step of the product against the previous commit's build
# (tools/build/libtowr_gpu_prev.so) on one box, then the step's in-kernel stamps
TAG=${1:-r05w}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4; do
  for V in "" prev; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 $L >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
timeout -k 10 200 python tools/stamps.py --fixed > gpurun_out/${TAG}_step.log 2>&1 || exit 1
cat gpurun_out/${TAG}_step.log
