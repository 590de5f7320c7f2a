#!/bin/bash
# Quick GPU iteration: parity tests, a short bench, one SQ-counter PMC pass.
# Usage: tools/gpu_ab.sh TAG
TAG=${1:-ab}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --no-host > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d gpurun_out/${TAG}_sq -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host > gpurun_out/${TAG}_sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
