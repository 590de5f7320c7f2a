#!/bin/bash
# GPU box: in-kernel phase stamps of the gait step (tools/stamps.py, experiment build tools/build/libtowr_gpu_stamps.so)
TAG=${1:-r05b}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_stamps_step.log 2>&1 || { cat gpurun_out/${TAG}_stamps_step.log; exit 1; }
timeout -k 10 200 python tools/stamps.py --only 2 > gpurun_out/${TAG}_stamps_fdisc.log 2>&1 || exit $?
timeout -k 10 200 python tools/stamps.py --only 0 > gpurun_out/${TAG}_stamps_dyn.log 2>&1 || exit $?
timeout -k 10 200 python tools/stamps.py --batch 1 > gpurun_out/${TAG}_stamps_b1.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_stamps_*.log
