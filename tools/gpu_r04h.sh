#!/bin/bash
# GPU-box: fixed-gait (headline and RotVec) same-box A/Bs of experiment builds. Usage: tools/gpu_r04h.sh TAG "lib1 ..."
TAG=${1:-r04h}; LIBS=$2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rotvec or fusion or anymal_trot or full_size or host_batch" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for LIB in "" $LIBS; do
    timeout -k 10 200 python tools/gait_ab.py --reps 100 --no-gait --batch 4096 ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
    timeout -k 10 200 python tools/gait_ab.py --reps 100 --no-gait --rotvec --batch 4096 ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_abrv.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log | grep -E "dynamic|step"
echo rotvec
grep -v amdgpu.ids gpurun_out/${TAG}_abrv.log | grep -E "dynamic|step"
