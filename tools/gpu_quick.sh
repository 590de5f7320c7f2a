#!/bin/bash
# GPU-box quick loop: parity tests, phase timing, short bench. Stops at the first failure.
# Usage: tools/gpu_quick.sh TAG
TAG=${1:-q}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/phase_timing.py > gpurun_out/${TAG}_phase.log 2>&1
rc=$?; echo "phase rc=$rc"; tail -6 gpurun_out/${TAG}_phase.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-host > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"
python tools/summ.py gpurun_out/${TAG}_bench.log 2>/dev/null || tail -c 1500 gpurun_out/${TAG}_bench.log
exit $rc
