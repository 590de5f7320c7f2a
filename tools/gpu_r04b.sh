#!/bin/bash
# GPU-box: gait parity, then same-box A/Bs of the gait steps (plain, + Torque) against saved builds, then kernel
# traces. Usage: tools/gpu_r04b.sh TAG "lib1 lib2 ..."
TAG=${1:-r04b}; LIBS=$2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for LIB in "" $LIBS; do
    timeout -k 10 200 python tools/gait_ab.py --reps 40 ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
    timeout -k 10 200 python tools/gait_ab.py --reps 40 --torque ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
for mode in "" "--torque" "--rotvec --batch 4096"; do
  name=$(echo "x$mode" | tr -dc 'a-z')
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$name -o run -- python tools/step_trace.py $mode > gpurun_out/${TAG}_$name.log 2>&1 || exit $?
done
