#!/bin/bash
# GPU box: the small kinds' one-level prologue (product) against round-4-style staging (TOWR_SPAN_SERIAL variant, built before the descriptor copies):
# headline step and per-kernel times, then stamps of the small kinds alone and of the step
TAG=${1:-r05t}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "batch" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in "" spanser; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 200 $L >> gpurun_out/${TAG}_ab.log 2>&1 || exit 1
  done
done
grep -E "small|step" gpurun_out/${TAG}_ab.log
timeout -k 10 200 python tools/stamps.py --fixed --only 4 > gpurun_out/${TAG}_misc.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py --fixed > gpurun_out/${TAG}_step.log 2>&1 || exit 1
cat gpurun_out/${TAG}_misc.log gpurun_out/${TAG}_step.log
