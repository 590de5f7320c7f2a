#!/bin/bash
# GPU box: 1 KB-aligned store trips per composer loop (product: FDISC; a0 none, a9 FDISC + TQDISC, a1u2 FDISC at 2 units):
# 3: both): gait and gait + Torque steps against the product, one box
TAG=${1:-r05ag}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for V in "" a0 a9 a1u2; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $3}') || exit 1
    echo "${V:-product} gait $g torque $t" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
