#!/bin/bash
# GPU box: the small kinds' per-thread x unit table (product) against the span-list walk (noxu), headline per-kernel and
# step times, one box; stamps of the small kinds alone
TAG=${1:-r05ak}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for V in "" noxu; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 $L 2>&1 | grep -E "small|step" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
