#!/bin/bash
# GPU box: same-box A/B of the composers' store depth (FDISC units, GsBlock units per lane): product (4, 4) vs variants
TAG=${1:-r05p}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for V in "" fu2 f1g1 f2g1 f4g2 f1g2; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    echo "${V:-product} gait $(timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $L 2>&1 | grep step | awk '{print $NF, $(NF-1)}') torque $(timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only --torque $L 2>&1 | grep step | awk '{print $(NF-1)}')" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
