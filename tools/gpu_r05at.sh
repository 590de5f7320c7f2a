#!/bin/bash
# GPU box: RotVec step, product (with / without the Dynamic overlap, TOWR_GPU_ROTVEC_OVERLAP) against round 4's build
TAG=${1:-r05at}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4; do
  a=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 300 --step-only 2>&1 | grep step | awk '{print $3}') || exit 1
  b=$(TOWR_GPU_ROTVEC_OVERLAP=0 timeout -k 10 200 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 300 --step-only 2>&1 | grep step | awk '{print $3}') || exit 1
  c=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 300 --step-only --lib tools/build/libtowr_gpu_base.so 2>&1 | grep step | awk '{print $3}') || exit 1
  h=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 --step-only 2>&1 | grep step | awk '{print $3}') || exit 1
  hb=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 --step-only --lib tools/build/libtowr_gpu_base.so 2>&1 | grep step | awk '{print $3}') || exit 1
  echo "rotvec product $a no-overlap $b base $c | headline product $h base $hb" >> gpurun_out/${TAG}_ab.log
done
cat gpurun_out/${TAG}_ab.log
