#!/bin/bash
# round-3 baseline on the GPU box: gait per-kernel times and a short bench (product build)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gait_ab.py --reps 30 > gpurun_out/r03a_gait.log 2>&1 || exit $?
timeout -k 10 300 python tools/gait_ab.py --reps 30 --no-gait --batch 4096 > gpurun_out/r03a_euler.log 2>&1 || exit $?
timeout -k 10 300 python tools/single_probe.py > gpurun_out/r03a_single.log 2>&1 && timeout -k 10 300 python tools/single_probe.py gait >> gpurun_out/r03a_single.log 2>&1 || exit $?
cat gpurun_out/r03a_gait.log gpurun_out/r03a_euler.log gpurun_out/r03a_single.log
