#!/bin/bash
# GPU-box: kernel traces of the gait steps (plain, + Torque) and the RotVec step, plus the round-3 library beside
# the product on the plain gait step. Usage: tools/gpu_r04t.sh TAG
TAG=${1:-r04t}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for mode in "" "--torque" "--rotvec --batch 4096"; do
  name=$(echo "x$mode" | tr -dc 'a-z')
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$name -o run -- python tools/step_trace.py $mode > gpurun_out/${TAG}_$name.log 2>&1 || exit $?
done
for i in 1 2; do
  for LIB in "" tools/build/libtowr_gpu_r04base.so tools/build/libtowr_gpu_r03.so; do
    timeout -k 10 200 python tools/gait_ab.py --reps 40 ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for LIB in "" tools/build/libtowr_gpu_miscfork.so tools/build/libtowr_gpu_r03.so; do
    timeout -k 10 200 python tools/gait_ab.py --reps 100 --no-gait --batch 4096 ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
