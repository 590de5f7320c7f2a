#!/bin/bash
# GPU-box: the -m gpu suite, then same-box A/Bs of the product against saved builds on every bench workload
# (headline, RotVec, gait, gait + Torque). Usage: tools/gpu_r04k.sh TAG "lib1 ..."
TAG=${1:-r04k}; LIBS=$2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for LIB in "" $LIBS; do
    for mode in "--no-gait --batch 4096 --reps 100" "--no-gait --rotvec --batch 4096 --reps 100" "--reps 40" "--torque --reps 40 --step-only"; do
      echo "== ${LIB:-product} $mode" >> gpurun_out/${TAG}_ab.log
      timeout -k 10 200 python tools/gait_ab.py $mode ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log | grep -E "^==|step|dynamic|small_kinds|force_disc"
