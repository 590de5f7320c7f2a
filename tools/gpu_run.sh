#!/bin/bash
# GPU-box driver: parity tests, a short bench, a rocprofv3 kernel-trace profile.
# Usage: tools/gpu_run.sh TAG [steps]
# Stops at the first GPU fault / abort / timeout (exit 124, 134, 137, 139); plain test failures
# (exit 1) do not stop the bench.
TAG=${1:-r}
STEPS=${2:-20}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_pytest.log
ok_rc $rc || exit $rc

timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 --cpu-seconds 10 > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python bench.py --steps $STEPS --warmup 3 --no-cpu --no-host > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/${TAG}_prof.log
find gpurun_out/${TAG}_prof -name "*stats*" | head
exit $rc
