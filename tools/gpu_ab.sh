#!/bin/bash
# A/B of the two output paths (direct HBM stores vs LDS-staged tile) + parity tests in both modes.
TAG=${1:-ab}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest_direct.log 2>&1
rc=$?; echo "pytest direct rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_direct.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TOWR_GPU_OUTPUT=lds timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest_lds.log 2>&1
rc=$?; echo "pytest lds rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_lds.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mode in direct lds; do
  TOWR_GPU_OUTPUT=$mode timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/${TAG}_bench_$mode.log 2>&1
  rc=$?; echo "bench $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
