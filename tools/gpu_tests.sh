#!/bin/bash
# GPU-box: the -m gpu suite only (optionally a -k selection), one process, stops at the first failure.
# Usage: tools/gpu_tests.sh TAG [pytest -k expression]
TAG=${1:-t}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$2" ]; then SEL=(-k "$2"); else SEL=(); fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${SEL[@]}" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/${TAG}_pytest.log
exit $rc
