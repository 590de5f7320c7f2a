#!/bin/bash
# A/B of the fork-join launch (TOWR_GPU_STREAMS = 1 serial .. 4) + parity tests with the default.
TAG=${1:-st}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for n in 1 2 4; do
  TOWR_GPU_STREAMS=$n timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --no-host > gpurun_out/${TAG}_bench_s$n.log 2>&1
  rc=$?; echo "bench streams=$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
