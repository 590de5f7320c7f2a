#!/bin/bash
# GPU box: the round-close run (tools/gpu_r05zz.sh), then the gait step's in-kernel stamps (the composers' phases)
TAG=${1:-r05zz}
cd "$(dirname "$0")/.."
tools/gpu_r05zz.sh $TAG || exit 1
timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_stamps_gait.log 2>&1 || exit 1
cat gpurun_out/${TAG}_stamps_gait.log
