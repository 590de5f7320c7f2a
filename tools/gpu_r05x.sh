#!/bin/bash
# GPU box: the slot-address source per tile type (TOWR_SLOT0_MASK variants) on the headline step, one box
TAG=${1:-r05x}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for V in "" s0none s0all prev; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 $L >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
