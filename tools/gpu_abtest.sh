#!/bin/bash
# A/B of two engine builds on one box: tools/build/libtowr_gpu_prev.so (A) vs the in-tree library (B),
# alternating bench runs (100 steps each, 3 rounds). Usage: tools/gpu_abtest.sh TAG
TAG=${1:-abt}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  TOWR_GPU_LIB=$PWD/tools/build/libtowr_gpu_prev.so timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu --no-host > gpurun_out/${TAG}_A$r.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu --no-host > gpurun_out/${TAG}_B$r.log 2>&1 || exit $?
done
python tools/summ.py gpurun_out/${TAG}_A*.log gpurun_out/${TAG}_B*.log
