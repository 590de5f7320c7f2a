#!/bin/bash
# GPU box: same-box A/B of the composers' store depth, more repetitions: product (4, 4), (1, 2), (1, 1), (2, 2)
TAG=${1:-r05q}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for V in "" f1g2 f1g1 fu2; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    echo "${V:-product} gait $(timeout -k 10 200 python tools/gait_ab.py --reps 100 --step-only $L 2>&1 | grep step | awk '{print $(NF-1)}') torque $(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $(NF-1)}')" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
