#!/bin/bash
# GPU box: in-kernel phase stamps of the headline step (fixed phase durations, B = 4096): the whole step, Dynamic alone,
# the small kinds alone
TAG=${1:-r05s}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py --fixed > gpurun_out/${TAG}_step.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py --fixed --only 0 > gpurun_out/${TAG}_dyn.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py --fixed --only 4 > gpurun_out/${TAG}_misc.log 2>&1 || exit 1
cat gpurun_out/${TAG}_*.log
