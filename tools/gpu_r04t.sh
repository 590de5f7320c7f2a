#!/bin/bash
# GPU-box: kernel traces of the gait steps (plain, + Torque) and the RotVec step, plus the round-3 library beside
# the product on the plain gait step. Usage: tools/gpu_r04t.sh TAG
TAG=${1:-r04t}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in "" "--torque" "--rotvec --batch 4096"; do
  name=$(echo "x$mode" | tr -dc 'a-z')
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$name -o run -- python tools/step_trace.py $mode > gpurun_out/${TAG}_$name.log 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 200 python tools/gait_ab.py --reps 40 >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  timeout -k 10 200 python tools/gait_ab.py --reps 40 --lib tools/build/libtowr_gpu_r03.so >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
