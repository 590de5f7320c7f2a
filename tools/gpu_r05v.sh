#!/bin/bash
# GPU box: headline step with the small kinds before / after Dynamic on the side stream (TOWR_GPU_MISC_FIRST)
TAG=${1:-r05v}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4; do
  a=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 --step-only 2>&1 | grep step) || exit 1
  b=$(TOWR_GPU_MISC_FIRST=1 timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 --step-only 2>&1 | grep step) || exit 1
  echo "last [$a] first [$b]" >> gpurun_out/${TAG}_ab.log
done
cat gpurun_out/${TAG}_ab.log
