#!/bin/bash
# GPU box: same-box A/B of the composers' store depth (16-byte units per lane before their stores: 4 product, 2, 8)
TAG=${1:-r05o}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for L in "" "--lib tools/build/libtowr_gpu_fu2.so" "--lib tools/build/libtowr_gpu_fu8.so"; do
    timeout -k 10 200 python tools/gait_ab.py --reps 40 $L 2>&1 | grep -v amdgpu.ids >> gpurun_out/${TAG}_ab.log || exit 1
    echo "torque ${L:-product} $(timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only --torque $L 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
