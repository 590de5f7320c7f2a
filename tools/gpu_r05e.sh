#!/bin/bash
TAG=${1:-r05e}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TOWR_GPU_GAIT_SCHED=pipe4 timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_stamps_pipe4.log 2>&1 || exit $?
TOWR_GPU_GAIT_SCHED=chain timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_stamps_chain.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_stamps_*.log
