#!/bin/bash
# GPU-box quick check: the -m gpu suite, the gait per-kernel figures and the B = 1 probes.
# Usage: tools/gpu_quick.sh TAG [gait_ab args...]
TAG=${1:-q}
shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gait_ab.py --reps 30 "$@" > gpurun_out/${TAG}_gait.log 2>&1
rc=$?; echo "gait rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_gait.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/single_probe.py gait > gpurun_out/${TAG}_single.log 2>&1
rc=$?; echo "single rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_single.log
exit $rc
