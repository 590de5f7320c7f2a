#!/bin/bash
# GPU-box round check: the -m gpu suite, the bench with the driver's flags, the gait / Euler per-kernel
# A/B figures and a rocprofv3 kernel-trace --stats pass of the bench. Stops at the first failing step.
# Usage: tools/gpu_round.sh TAG [--no-tests]
TAG=${1:-r}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gait_ab.py --reps 30 > gpurun_out/${TAG}_gait.log 2>&1
rc=$?; echo "gait rc=$rc"; cat gpurun_out/${TAG}_gait.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu --no-host > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find gpurun_out/${TAG}_prof -name "*stats*"
exit $rc
