#!/bin/bash
# A/B of an engine environment switch on one box: parity tests with the default, then alternating
# bench runs with VAR set to each value (3 rounds). Usage: tools/gpu_env_ab.sh TAG VAR "v1 v2 ..."
TAG=${1:-env}; VAR=$2; VALS=$3
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu --no-host > gpurun_out/${TAG}_${v}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $VAR=$v rc=$rc"; exit $rc; }
  done
done
for v in $VALS; do echo "== $VAR=$v"; python tools/summ.py gpurun_out/${TAG}_${v}_*.log; done
