#!/bin/bash
# GPU-box: per-kernel times of the gait batch for the product and the experiment builds
# (tools/build/libtowr_gpu_{nozero,nostore,noeval}.so), then WRITE_SIZE / FETCH_SIZE passes over the
# product's gait batch. Usage: tools/gpu_gait_probe.sh TAG
TAG=${1:-gp}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/gait_ab.py > gpurun_out/${TAG}_ab.log 2>&1 || exit $?
for v in nozero nostore noeval; do
  [ -f tools/build/libtowr_gpu_$v.so ] || continue
  timeout -k 10 120 python tools/gait_ab.py --lib tools/build/libtowr_gpu_$v.so >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
done
cat gpurun_out/${TAG}_ab.log
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/${TAG}_$c -o run -- \
      python3 tools/gait_ab.py --reps 3 > gpurun_out/${TAG}_$c.log 2>&1 || exit $?
done
python3 tools/pmc_summ.py gpurun_out/${TAG}_WRITE_SIZE gpurun_out/${TAG}_FETCH_SIZE 2>&1 | tail -30
exit 0
