#!/bin/bash
# Same-box A/B of the gait step: an experiment / baseline build under tools/build against the product
# library, alternating. Usage: tools/gpu_ab_lib.sh TAG LIB [rounds] [gait_ab args...]
TAG=${1:-ab}; LIB=$2; N=${3:-2}
shift 3
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq $N); do
  timeout -k 10 200 python tools/gait_ab.py --reps 40 --lib $LIB "$@" >> gpurun_out/${TAG}.log 2>&1 || exit $?
  timeout -k 10 200 python tools/gait_ab.py --reps 40 "$@" >> gpurun_out/${TAG}.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/${TAG}.log
