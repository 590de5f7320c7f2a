#!/bin/bash
# GPU box: kernel trace + stamps of the gait + Torque step (chain schedule)
TAG=${1:-r05n}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trq -o run -- python tools/step_trace.py --torque > gpurun_out/${TAG}_trq.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py --torque > gpurun_out/${TAG}_st_t.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${TAG}_st_t.log | sed 's/_ZN2tg12_GLOBAL__N_1[0-9]*//; s/EvNS_7KParams.*E:/:/' | cut -c1-220
