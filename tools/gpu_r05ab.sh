#!/bin/bash
# GPU box: kernel traces of the gait + Torque and the plain gait steps (tools/step_trace.py) for tools/step_timeline.py
TAG=${1:-r05ab}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tq -o run -- python3 tools/step_trace.py --torque --steps 30 > gpurun_out/${TAG}_tq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_g -o run -- python3 tools/step_trace.py --steps 30 > gpurun_out/${TAG}_g.log 2>&1 || exit 1
ls gpurun_out/${TAG}_tq gpurun_out/${TAG}_g
