#!/bin/bash
# GPU box: problems per composer block (TOWR_GS_GROUP: product 2, g1, g4):
# gait, gait + Torque and headline steps, one box
TAG=${1:-r05ai}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for V in "" g1 g4; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $3}') || exit 1
    h=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    echo "${V:-product} gait $g torque $t headline $h" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
