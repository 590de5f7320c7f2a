#!/bin/bash
# GPU-box session script of round 4: a -m gpu selection, then per-kernel gait figures (product, + Torque) and an
# optional experiment builds beside the product. Usage: tools/gpu_r04.sh TAG "pytest -k expr" ["lib1 lib2 ..."]
TAG=${1:-r04}; SEL=$2; LIBS=$3
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$SEL" > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/${TAG}_pytest.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python tools/gait_ab.py --reps 40 --no-gait --rotvec --batch 4096 >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python tools/gait_ab.py --reps 40 >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
  timeout -k 10 200 python tools/gait_ab.py --reps 40 --torque >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
  for LIB in $LIBS; do
    timeout -k 10 200 python tools/gait_ab.py --reps 40 --lib $LIB >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
    timeout -k 10 200 python tools/gait_ab.py --reps 40 --torque --lib $LIB >> gpurun_out/${TAG}_gait.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_gait.log
